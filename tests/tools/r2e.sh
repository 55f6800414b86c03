cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u tests/kexp/stem_exp.py 2>&1 | tee gpurun_out/r2e_stemexp.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2e_prof -o run -- python3 $R/tests/kexp/stem_exp.py > $R/gpurun_out/r2e_prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA -d $R/gpurun_out/r2e_pmc1 -o run --output-format csv -- python3 $R/tests/kexp/stem_exp.py > $R/gpurun_out/r2e_pmc1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $R/gpurun_out/r2e_pmc2 -o run --output-format csv -- python3 $R/tests/kexp/stem_exp.py > $R/gpurun_out/r2e_pmc2.log 2>&1
