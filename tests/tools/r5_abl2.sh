#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OLDPWD/gpurun_out/r5_counters.txt 2>&1
cd $OLDPWD
timeout -k 10 900 python -u tests/tools/big_abl.py "" abl5 abl30 abl22 abl7 > gpurun_out/r5_big_abl2.txt 2>&1 || exit $?
timeout -k 10 300 python -u tests/tools/layer_times.py --clock --out gpurun_out/r5_layer_times_clock.json > gpurun_out/r5_layer_times_clock.log 2>&1 || exit $?
head -30 gpurun_out/r5_layer_times_clock.log
