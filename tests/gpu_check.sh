#!/bin/bash
# One GPU session: op + parity tests, smoke, bench, kernel-trace profile.
# Usage: tests/gpu_check.sh TAG [--no-tests]
# Every GPU step has its own time limit; the script stops at the first step that aborts,
# faults or times out (exit status > 1), so nothing more runs on a sick GPU.
TAG=${1:-run}
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_bad() {  # $1 = step name, $2 = status
  if [ "$2" -gt 1 ]; then echo "$1 ended with status $2: stopping"; exit "$2"; fi
}
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
  rc=$?
  echo "tests_rc=$rc"; grep -E "passed|failed|error" gpurun_out/tests_$TAG.log | tail -3
  stop_if_bad tests $rc
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 gpurun_out/smoke_$TAG.log; stop_if_bad smoke $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -1 gpurun_out/bench_$TAG.log; stop_if_bad bench $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run \
  --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --fp32-steps 0 \
  > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof_rc=$rc"; tail -1 gpurun_out/prof_$TAG.log
