#!/bin/bash
# packed-fp32 head / maxpool BN-backward passes: their op tests, then the in-step A/B against
# the previous ops.hip build (libpcms_hip_opsold.so) with the bench's final loss compared
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6o}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py -m gpu -v --timeout 200 --timeout-method thread -k "head or pool or bn" > gpurun_out/${TAG}_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_ops.log | tail -3
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 bash tests/tools/r6_libab.sh ${TAG} prod opsold
python3 -c "
import json
for v in ('prod','opsold'):
    print(v, [json.load(open(f'gpurun_out/${TAG}_{v}_{r}.json'))['final_loss'] for r in (1,2,3)])"
