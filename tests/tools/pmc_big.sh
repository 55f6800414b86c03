#!/bin/bash
# PMC passes over the big-box conv (tests/tools/big_one.py), product and variant libraries.
# Usage: pmc_big.sh TAG "libsuffix ..." [shape]
cd "$(dirname "$0")/../.."
R=$PWD
TAG=$1; LIBS=$2; SH=${3:-0}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE GRBM_TA_BUSY"
P2="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
P3="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
P4="TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum"
for lib in $LIBS; do
  if [ "$lib" = product ]; then unset PCMS_LIB; else export PCMS_LIB=$R/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_$lib.so; fi
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/${TAG}_${lib}_p$i -o pmc -- python3 $R/tests/tools/big_one.py $SH 5 > $R/gpurun_out/${TAG}_${lib}_p$i.log 2>&1 || { echo "pmc $lib p$i rc=$?"; exit 1; }
  done
done
echo pmc done
