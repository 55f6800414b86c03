#!/bin/bash
# One GPU session: op tests, parity tests, bench, kernel profile.  Usage: tests/gpu_check.sh TAG
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -q -p no:cacheprovider > gpurun_out/tests_$TAG.log 2>&1
rc=$?
echo "tests_rc=$rc"; tail -3 gpurun_out/tests_$TAG.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
rc=$?
echo "bench_rc=$rc"; tail -1 gpurun_out/bench_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --kernel-reps 5 > gpurun_out/prof_$TAG.log 2>&1
echo "prof_rc=$?"
