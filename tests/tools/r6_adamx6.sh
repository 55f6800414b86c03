#!/bin/bash
# fp32 build's fused Adam with batched loads: its op tests, then a kernel trace of the fp32
# bench (adam_pack_conv3_x6_kernel's time against profiles/r6_step_kernel_stats_final.csv).
# Record: profiles/r6_adam_x6_batched.txt
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_step_variants.py -m gpu -x -v -k "adam" --timeout 200 --timeout-method thread > gpurun_out/r6_adamx6_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r6_adamx6_tests.log
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
R=$PWD
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6_adamx6_prof -o run --output-format csv -- python3 $R/bench.py --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline --fp32-steps 0 --kernel-reps 2 > $R/gpurun_out/r6_adamx6_prof.log 2>&1)
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/r6_adamx6_prof.log
[ $rc -eq 0 ] || exit $rc
# the input-pack skip ablation (profiles/r6_pack_input_skip_ab.txt), ABBA rounds
timeout -k 10 400 python -u tests/tools/step_ab.py --rounds 8 --steps 10 --variants base,nopack > gpurun_out/r6s2_nopack_abba.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -2 gpurun_out/r6s2_nopack_abba.txt
