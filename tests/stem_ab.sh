#!/bin/bash
# A/B of the stem forward variants (PCMS_STEM_FWD_PIPE) + stem parity tests.  Test tooling.
TAG=${1:-ab}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k stem -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/stem_tests_$TAG.log 2>&1
rc=$?; echo "tests_rc=$rc"; grep -E "passed|failed" gpurun_out/stem_tests_$TAG.log | tail -2; [ $rc -gt 1 ] && exit $rc
for v in 0 2 0 2; do
  PCMS_STEM_FWD_PIPE=$v timeout -k 10 120 python -u tests/bench_stem.py fwd 50 > gpurun_out/stem_ab_$TAG.$v.log 2>&1
  rc=$?; echo "pipe=$v rc=$rc $(grep 'stem fwd' gpurun_out/stem_ab_$TAG.$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
