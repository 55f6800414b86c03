#!/bin/bash
# One GPU call: the GPU test suite, then (only if no crash/timeout) the bench and a rocprof
# kernel summary.  Every GPU step has its own time limit; a crash / abort / timeout ends
# the script (exit codes 124/134/137/139 or a signal), plain test failures (rc 1) do not.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-run}
PHASES=${PHASES:-tests bench prof}
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
if [[ " $PHASES " == *" tests "* ]]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
  ok $rc || exit $rc
fi
if [[ " $PHASES " == *" bench "* ]]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json
  [ $rc -eq 0 ] || exit $rc
fi
if [[ " $PHASES " == *" prof "* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/gpurun_out/${TAG}_prof -o prof -- \
    python3 $OLDPWD/bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-steps 0 ${BENCH_ARGS:-} > $OLDPWD/gpurun_out/${TAG}_prof.log 2>&1
  rc=$?; echo "prof rc=$rc"
  exit $rc
fi
