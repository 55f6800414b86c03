#!/bin/bash
# fp32 build: x6 forward MFMA order A/B -- fp32 op / parity tests, kernel trace, in-step bench
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6so}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py tests/test_determinism.py -m gpu -v --timeout 400 --timeout-method thread -k "fp32 or x6 or conv3 or parity" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
bash tests/tools/r6_x6abl.sh ${TAG}k sord0 || exit 1
BENCH_ARGS="--precision fp32 --steps 6 --warmup 2" ROUNDS=2 bash tests/tools/r6_libab.sh ${TAG}b prod sord0
