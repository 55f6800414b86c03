#!/bin/bash
# one-launch ConvTranspose split / bias reduction: convT op tests (bit-identity vs the separate
# launches, fp64 bars), the kernel-trace A/B and the in-step A/B against libpcms_hip_ctold.so
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6c}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -v --timeout 200 --timeout-method thread -k "convt" > gpurun_out/${TAG}_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_ops.log | tail -3
[ $rc -eq 0 ] || exit $rc
bash tests/tools/r6_ktrace_ab.sh ${TAG}k ctold convt_reduce_fused convt_group_sum convt_wgrad_reduce convt_bias_reduce convt_wgrad128 || exit 1
ROUNDS=3 bash tests/tools/r6_libab.sh ${TAG}b prod ctold
