# big-box persistent kernel: op tests, then kernel timings (level 0/1 shapes)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "big_box or conv3_fwd or dual" > gpurun_out/r2n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2n_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/bench_kernels.py --only fwd,dgrad --reps 20 > gpurun_out/r2n_kern.log 2>&1
rc=$?; cat gpurun_out/r2n_kern.log; exit $rc
