#!/bin/bash
# general conv XCD-aware grid: conv op tests, same-box A/B against ab/r5a, layer times
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5x}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "conv3 or split" > gpurun_out/${TAG}_ops.log 2>&1 || { tail -30 gpurun_out/${TAG}_ops.log; exit 1; }
tail -2 gpurun_out/${TAG}_ops.log
bash tests/tools/tree_ab.sh ${TAG} 2 ab/r5a . || exit $?
timeout -k 10 300 python -u tests/tools/layer_times.py --clock --out gpurun_out/${TAG}_layers.json > gpurun_out/${TAG}_layers.log 2>&1 || exit $?
echo done
