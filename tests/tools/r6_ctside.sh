#!/bin/bash
# ConvT weight gradient on the side stream: its bit-identity test, then the in-step A/B (ABBA)
# and a kernel trace with it on.  Record: profiles/r6_convt_wgrad_side_ab.txt
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_step_variants.py -m gpu -x -v -k "convt_wgrad_side" --timeout 200 --timeout-method thread > gpurun_out/r6_ctside_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r6_ctside_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tests/tools/step_ab.py --rounds 8 --steps 10 --variants base,ctside > gpurun_out/r6_ctside_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -2 gpurun_out/r6_ctside_ab.txt
