cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u tests/kexp/stem_exp.py 2>&1 | tee gpurun_out/r2f_stemexp.log || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2f_prof -o run -- python3 $R/tests/kexp/stem_exp.py > $R/gpurun_out/r2f_prof.log 2>&1
