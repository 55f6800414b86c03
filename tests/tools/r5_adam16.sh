#!/bin/bash
# fused Adam writing the pack16 forms: parity tests, then same-box A/B against the previous tree
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-adam16}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_step_variants.py tests/test_gpu_configs.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash tests/tools/tree_ab.sh ${TAG} 3 ab/r5b . --steps 20 --warmup 5
