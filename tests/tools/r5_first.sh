#!/bin/bash
# Round 5, first GPU call: the clock probe checked against in-kernel clocks, the full bench on
# the working tree (with the new clock fields), then the round-3 vs round-4 final trees
# alternated on the same box.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
{ nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python -c "import os; print(len(os.sched_getaffinity(0)))"; } > gpurun_out/r5_cpuinfo.txt 2>&1
timeout -k 10 180 python -u tests/tools/clock_check.py > gpurun_out/r5_clock_check.txt 2>&1 || exit $?
cat gpurun_out/r5_clock_check.txt | head -60
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench_v0.json 2> gpurun_out/r5_bench_v0.err || exit $?
cat gpurun_out/r5_bench_v0.json
bash tests/tools/tree_ab.sh r5_r3r4 2 ab/r4 ab/r3
