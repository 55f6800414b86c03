#!/bin/bash
# one-launch weight-gradient split reduction: op tests (bit-identity vs the two-stage pair, fp64
# bars), the in-step A/B, then per-launch layer times with the product settings
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6w}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "wgrad" > gpurun_out/${TAG}_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_ops.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tests/tools/step_ab.py --rounds 4 --steps 10 --variants wred1,wred0 > gpurun_out/${TAG}_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 gpurun_out/${TAG}_ab.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/tools/layer_times.py --out gpurun_out/${TAG}_lt.json > gpurun_out/${TAG}_lt.log 2>&1
echo "lt rc=$?"
