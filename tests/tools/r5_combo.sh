#!/bin/bash
# conv + wgrad op tests, wgrad ablation (product vs no-staging), level-2 / level-3 standalone
# timings, same-box tree A/B against ab/r5a
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5c}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_blocks.py -k "wgrad or bnin or fwd16 or dgrad16 or conv16 or four_deep" > gpurun_out/${TAG}_ops.log 2>&1 || { tail -30 gpurun_out/${TAG}_ops.log; exit 1; }
tail -1 gpurun_out/${TAG}_ops.log
timeout -k 10 400 python -u tests/tools/wgrad_abl.py product w2 > gpurun_out/${TAG}_wabl.log 2>&1 || { tail -20 gpurun_out/${TAG}_wabl.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_wabl.log | grep 'round": 1' | cut -c1-150
timeout -k 10 300 python -u tests/tools/deep_ab.py > gpurun_out/${TAG}_deep.log 2>&1 || { tail -20 gpurun_out/${TAG}_deep.log; exit 1; }
grep k16_4 gpurun_out/${TAG}_deep.log | cut -c1-150
timeout -k 10 300 python -u tests/tools/deep3_ab.py > gpurun_out/${TAG}_deep3.log 2>&1 || { tail -20 gpurun_out/${TAG}_deep3.log; exit 1; }
grep k16 gpurun_out/${TAG}_deep3.log | cut -c1-150
bash tests/tools/tree_ab.sh ${TAG} 2 ab/r5a . || exit $?
echo done
