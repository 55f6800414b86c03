cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tests/kexp/stem_exp.py 2>&1 | grep -v "^wg mode\|read_stream" | tee gpurun_out/r2g_stemexp.log
