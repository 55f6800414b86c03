#!/bin/bash
# Round-6 second session, end: the whole evidence set of r6_final.sh on the final binary, then the
# per-launch layer times of the bench workload (plain and with per-launch clocks).
# Records: profiles/r6_*_final_s2*, profiles/r6_layer_times_final.json, r6_layer_times_final_clock.json
cd "$(dirname "$0")/../.."
bash tests/tools/r6_final.sh ${1:-r6s2f} || exit $?
timeout -k 10 300 python -u tests/tools/layer_times.py --steps 3 --out gpurun_out/r6s2f_layers.json > gpurun_out/r6s2f_layers.log 2>&1
rc=$?; echo "layers rc=$rc"; tail -2 gpurun_out/r6s2f_layers.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/tools/layer_times.py --steps 3 --clock --out gpurun_out/r6s2f_layers_clock.json > gpurun_out/r6s2f_layers_clock.log 2>&1
rc=$?; echo "layers clock rc=$rc"; tail -2 gpurun_out/r6s2f_layers_clock.log
