#!/bin/bash
# wgrad BNIN apply spread over k-steps: bit-identity tests, same-box A/B, layer times
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-bnin}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "bnin or wgrad" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
bash tests/tools/tree_ab.sh ${TAG} 3 ab/r5c . --steps 20 --warmup 5 || exit $?
timeout -k 10 300 python -u tests/tools/layer_times.py --clock --out gpurun_out/${TAG}_layers.json > gpurun_out/${TAG}_layers.log 2>&1 || exit $?
grep -E "wgrad_bnin|sum of" gpurun_out/${TAG}_layers.log
