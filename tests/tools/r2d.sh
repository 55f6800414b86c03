cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tests/kexp/stem_exp.py 2>&1 | tee gpurun_out/r2d_stemexp.log || exit $?
timeout -k 10 300 python -u -m pytest tests/test_step_variants.py tests/test_gpu_ops.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r2d_tests.log 2>&1; tail -5 gpurun_out/r2d_tests.log
