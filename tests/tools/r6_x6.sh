#!/bin/bash
# fp32 build weight gradient: the x6 op tests, the fp32 parity / determinism tests, then the
# in-step A/B (synchronous staging vs the LDS-DMA box stream) of the fp32 build
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6x6}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "x6 or (conv3_wgrad and not k16 and not many)" > gpurun_out/${TAG}_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; tail -3 gpurun_out/${TAG}_ops.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tests/tools/step_ab.py --precision fp32 --rounds 3 --steps 4 --variants x6dma,x6sync \
  > gpurun_out/${TAG}_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -4 gpurun_out/${TAG}_ab.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_determinism.py tests/test_gpu_configs.py -m gpu -v \
  --timeout 400 --timeout-method thread -k "fp32" > gpurun_out/${TAG}_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/${TAG}_parity.log | tail -12
