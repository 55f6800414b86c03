mkdir -p gpurun_out/pmc_big && export TMPDIR=/tmp
B="python tests/bench_kernels.py --names inc.conv3 --only fwdplain --reps 3"
timeout -s KILL 90 rocprofv3 -L > gpurun_out/pmc_big/avail.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY -d gpurun_out/pmc_big/g1 -o run --output-format csv -- $B > gpurun_out/pmc_big/g1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM -d gpurun_out/pmc_big/g2 -o run --output-format csv -- $B > gpurun_out/pmc_big/g2.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -d gpurun_out/pmc_big/g3 -o run --output-format csv -- $B > gpurun_out/pmc_big/g3.log 2>&1 || exit $?
