#!/bin/bash
# SQ / TA counters of the bf16 weight gradient at levels 0, 1, 3 (one --pmc pass per level).
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
O=$R/gpurun_out/pmc_wgrad_sq
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS TA_BUSY_avr GRBM_GUI_ACTIVE"
for lev in 0 1 3; do
  (cd /tmp && WGRAD_LEVEL=$lev timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc $C -d $O/l$lev -o run --output-format csv -- python3 $R/tests/kexp/wgrad_l0.py > $O/l$lev.log 2>&1) || exit $?
done
for lev in 0 1 3; do
  echo "== level $lev"
  python3 $R/tests/pmc_summary.py $(find $O/l$lev -name '*counter_collection.csv') --kernel conv3_wgrad_kernel
done
for lev in 0 1 3; do
  echo "== level $lev duration (ns)"
  grep conv3_wgrad_kernel $(find $O/l$lev -name '*kernel_stats.csv') | cut -d, -f1-5
done
