#!/bin/bash
# HBM traffic of the stem kernels (roofline "traffic"): FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes over tests/bench_stem.py (test tooling), summarised into $1 (JSON).
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
O=$R/gpurun_out/pmc_traffic
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
B="python3 $R/tests/bench_stem.py both 5"
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1) || exit $?
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B > $O/write.log 2>&1) || exit $?
python3 tests/kexp/stem_traffic.py $O ${1:-gpurun_out/stem_traffic.json}
