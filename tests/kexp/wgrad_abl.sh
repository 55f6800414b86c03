#!/bin/bash
# conv3 wgrad ablations (test tooling): 4096 no staging, 8192 no MFMA, 16384 no atomic flush
set -o pipefail
B="tests/bench_kernels.py --only wgrad --reps 10"
echo "== product"; timeout -k 10 200 python -u $B || exit $?
for a in 4096 8192 16384; do
  echo "== abl$a"; PCMS_LIB=tests/kexp/libpcms_abl$a.so timeout -k 10 200 python -u $B --names conv3 || exit $?
done
