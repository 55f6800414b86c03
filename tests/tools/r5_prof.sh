#!/bin/bash
# per-launch layer times with clocks + a rocprofv3 kernel trace of the bench
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5p}
timeout -k 10 300 python -u tests/tools/layer_times.py --clock --out gpurun_out/${TAG}_layers.json > gpurun_out/${TAG}_layers.log 2>&1 || exit $?
head -14 gpurun_out/${TAG}_layers.log
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_prof -o prof -- \
  python3 $R/bench.py --steps 7 --warmup 3 --no-cpu-baseline --fp32-steps 0 > $R/gpurun_out/${TAG}_prof.log 2>&1 || exit $?
echo prof ok
