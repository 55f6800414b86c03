#!/bin/bash
# 16x16x32 big-box kernel: its op tests, then (if green) the big-box timing vs the 32x32x16 one
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v -m gpu -k "fwd16 or dgrad16 or conv16 or big_box or bnin" --timeout 120 --timeout-method thread > gpurun_out/r5_b16_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r5_b16_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tests/tools/big_abl.py "" k16 > gpurun_out/r5_big_b16_ab.txt 2>&1 || exit $?
cat gpurun_out/r5_big_b16_ab.txt
