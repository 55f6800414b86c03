#!/bin/bash
# K16 weight gradient: op tests, ablation/A-B (16x16x32 vs 32x32x16, staging / MFMA ablations), tree A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5w}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_blocks.py -k "wgrad or bnin" > gpurun_out/${TAG}_ops.log 2>&1 || { tail -30 gpurun_out/${TAG}_ops.log; exit 1; }
tail -1 gpurun_out/${TAG}_ops.log
timeout -k 10 500 python -u tests/tools/wgrad_abl.py ${ABL:-"" w2 w4} > gpurun_out/${TAG}_abl.log 2>&1 || { tail -20 gpurun_out/${TAG}_abl.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_abl.log | cut -c1-150
bash tests/tools/tree_ab.sh ${TAG} 2 ab/r5a . || exit $?
echo done
