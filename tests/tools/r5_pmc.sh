#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tests/tools/layer_times.py --clock --out gpurun_out/r5_layer_times_clock.json > gpurun_out/r5_layer_times_clock.log 2>&1 || exit $?
head -12 gpurun_out/r5_layer_times_clock.log
bash tests/tools/pmc_big.sh r5pmc "product abl1" 0
