# PMC passes over the level-0 64->64 conv (fwd big-box, dgrad, wgrad): one rocprofv3 run per
# counter group (hardware limits per pass), summaries by tests/pmc_summary.py.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/pmc_conv; mkdir -p $O; export TMPDIR=/tmp
R=$PWD
B="python3 $R/tests/bench_kernels.py --names ${NAMES:-inc.conv3} --only ${ONLY:-fwdplain,wgrad} --reps 3"
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
         "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE TCP_TCC_READ_REQ_sum TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $G -d $R/$O/g$i -o run --output-format csv -- $B > $R/$O/g$i.log 2>&1) || exit $?
done
for K in ${KERNELS:-conv3_fwd_big conv3_wgrad_kernel}; do
  echo "== $K"
  python3 tests/pmc_summary.py $(find $O -name "*counter_collection.csv") --kernel $K
done
