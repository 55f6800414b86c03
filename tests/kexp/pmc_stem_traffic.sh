#!/bin/bash
# HBM traffic of the stem kernels (roofline "traffic"): FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes over tests/bench_stem.py (test tooling).
set -o pipefail
mkdir -p gpurun_out/pmc_traffic
export TMPDIR=/tmp
B="python tests/bench_stem.py both 5"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_traffic/fetch -o run --output-format csv -- $B > gpurun_out/pmc_traffic/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_traffic/write -o run --output-format csv -- $B > gpurun_out/pmc_traffic/write.log 2>&1 || exit $?
