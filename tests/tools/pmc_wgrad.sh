#!/bin/bash
# PMC passes over one weight-gradient shape (tests/tools/wgrad_one.py), one pass per run.
# Usage: pmc_wgrad.sh TAG [shape]
cd "$(dirname "$0")/../.."
R=$PWD
TAG=$1; SH=${2:-0}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="FETCH_SIZE"
P2="WRITE_SIZE"
P3="TCC_HIT_sum TCC_MISS_sum"
P4="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/${TAG}_p$i -o pmc -- python3 $R/tests/tools/wgrad_one.py $SH 5 > $R/gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pmc p$i rc=$?"; exit 1; }
done
cd $R && python3 tests/tools/pmc_table.py gpurun_out/${TAG} conv3_wgrad_kernel
