#!/bin/bash
# Round 5: clock probe re-check (CU-matched stamps), big-box ablations with clocks, per-launch
# layer times with clocks.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 180 python -u tests/tools/clock_check.py > gpurun_out/r5_clock_check2.txt 2>&1 || exit $?
timeout -k 10 900 python -u tests/tools/big_abl.py "" abl1 abl2 abl4 abl8 abl16 abl11 abl20 > gpurun_out/r5_big_abl.txt 2>&1 || exit $?
timeout -k 10 300 python -u tests/tools/layer_times.py --clock --out gpurun_out/r5_layer_times_clock.json > gpurun_out/r5_layer_times_clock.log 2>&1 || exit $?
head -40 gpurun_out/r5_layer_times_clock.log
