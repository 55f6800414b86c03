cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "stem" -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2h_tests.log 2>&1; tail -3 gpurun_out/r2h_tests.log
timeout -k 10 200 python -u tests/kexp/stem_exp.py 2>&1 | grep -v "^wg mode\|read_stream\|fwd ws" | tee gpurun_out/r2h_stemexp.log
