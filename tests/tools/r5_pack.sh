#!/bin/bash
# fragment-major bf16 pack: conv op tests + golden parity, then the big-box A/B vs the old pack
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5_pack_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5_pack_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u tests/tools/big_abl.py "" oldpack > gpurun_out/r5_big_pack_ab.txt 2>&1 || exit $?
cat gpurun_out/r5_big_pack_ab.txt
