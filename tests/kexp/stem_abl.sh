#!/bin/bash
# Stem kernel ablations + HBM calibration on the box (test tooling).
# abl1: fwd without MFMA, abl2: fwd without stores, abl4: fwd without halo prefetch,
# abl8: wgrad without MFMA, abl16: wgrad without staging.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tests/kexp/calib.py || exit $?
for rep in 1 2; do
  echo "== product run $rep"
  timeout -k 10 120 python -u tests/bench_stem.py both 30 || exit $?
done
for a in 1 2 4 8 16; do
  echo "== abl$a"
  PCMS_LIB=tests/kexp/libpcms_abl$a.so timeout -k 10 120 python -u tests/bench_stem.py both 30 || exit $?
done
