#!/bin/bash
# HBM traffic of the level-0 ConvTranspose forward, stream vs LDS kernel (test tooling):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes over tests/tools/convt_ab.py.
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
O=$R/gpurun_out/pmc_convt
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/tests/tools/convt_ab.py > $O/fetch.log 2>&1) || exit $?
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/tests/tools/convt_ab.py > $O/write.log 2>&1) || exit $?
for k in convt_fwd_stream_kernel "convt_lds_kernel<true"; do
  echo "== $k"
  python3 $R/tests/pmc_summary.py $(find $O/fetch $O/write -name '*counter_collection.csv') --kernel "$k"
done
