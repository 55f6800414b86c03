#!/bin/bash
# HBM traffic of the level-0 bf16 weight gradient (FETCH_SIZE / WRITE_SIZE, separate passes).
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
O=$R/gpurun_out/pmc_wgrad
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/tests/kexp/wgrad_l0.py > $O/fetch.log 2>&1) || exit $?
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/tests/kexp/wgrad_l0.py > $O/write.log 2>&1) || exit $?
python3 $R/tests/pmc_summary.py $(find $O/fetch $O/write -name '*counter_collection.csv') --kernel conv3_wgrad_kernel
python3 $R/tests/pmc_summary.py $(find $O/fetch $O/write -name '*counter_collection.csv') --kernel wgrad_reduce
