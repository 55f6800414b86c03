#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, kernel-trace only) for a command.
# Usage: tests/pmc_run.sh TAG -- python tests/bench_stem.py fwd 5
TAG=$1; shift; [ "$1" == "--" ] && shift
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU" \
           "SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "FETCH_SIZE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}/g$i -o run --output-format csv -- "$@" \
    > gpurun_out/pmc_${TAG}_g$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo "pmc ok"
