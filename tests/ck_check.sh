export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -k "checkpointing or True" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_ck2.log 2>&1
rc=$?; echo "tests_rc=$rc"; grep -E "passed|failed|Error" gpurun_out/tests_ck2.log | tail -5
