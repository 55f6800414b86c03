#!/bin/bash
# general conv tests, deep_ab (level-2 shapes general vs 16x16x32), same-box tree A/B, layer times
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5d}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "conv3 or split or fwd16 or dgrad16 or conv16" > gpurun_out/${TAG}_ops.log 2>&1 || { tail -30 gpurun_out/${TAG}_ops.log; exit 1; }
tail -2 gpurun_out/${TAG}_ops.log
timeout -k 10 300 python -u tests/tools/deep_ab.py > gpurun_out/${TAG}_deep.log 2>&1 || { tail -20 gpurun_out/${TAG}_deep.log; exit 1; }
cat gpurun_out/${TAG}_deep.log | grep -v amdgpu.ids
bash tests/tools/tree_ab.sh ${TAG} 2 ab/r5a . || exit $?
timeout -k 10 300 python -u tests/tools/layer_times.py --clock --out gpurun_out/${TAG}_layers.json > gpurun_out/${TAG}_layers.log 2>&1 || exit $?
echo done
