#!/bin/bash
# Selected GPU tests (-k $2) + short bench + kernel-trace profile.  Test tooling.
TAG=${1:-q}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "$2" -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/qtests_$TAG.log 2>&1
rc=$?; echo "tests_rc=$rc"; grep -E "passed|failed" gpurun_out/qtests_$TAG.log | tail -2; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/qbench_$TAG.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -1 gpurun_out/qbench_$TAG.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run \
  --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "prof_rc=$?"
