#!/bin/bash
# level-3 16x16x32 split-K form: op tests, standalone A/B, tree A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5l}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "fwd16 or dgrad16 or conv16 or four_deep" > gpurun_out/${TAG}_ops.log 2>&1 || { tail -30 gpurun_out/${TAG}_ops.log; exit 1; }
tail -1 gpurun_out/${TAG}_ops.log
timeout -k 10 300 python -u tests/tools/deep3_ab.py > gpurun_out/${TAG}_ab.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_ab.log | cut -c1-160
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_configs.py -k "bf16_build" > gpurun_out/${TAG}_cfg.log 2>&1 || { tail -30 gpurun_out/${TAG}_cfg.log; exit 1; }
tail -1 gpurun_out/${TAG}_cfg.log
bash tests/tools/tree_ab.sh ${TAG} 2 ab/r5a . || exit $?
echo done
