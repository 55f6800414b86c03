cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_determinism.py tests/test_step_variants.py tests/test_dp_gpu.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/r2c_tests.log 2>&1; rc=$?; tail -15 gpurun_out/r2c_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tests/kexp/stem_exp.py 2>&1 | tee gpurun_out/r2c_stemexp.log || exit $?
timeout -k 10 120 python -u tests/kexp/calib.py 2>&1 | tee gpurun_out/r2c_calib.log
