#!/bin/bash
# Big-box conv forward ablations (test tooling): 32 no in-chunk halo DMA, 64 no B loads,
# 128 no vm waits, 96 neither DMA nor B loads.
set -o pipefail
mkdir -p gpurun_out
B="tests/bench_kernels.py --names inc.conv3 --only fwdplain,dgrad --reps 10"
echo "== product"; timeout -k 10 120 python -u $B || exit $?
for a in 96 352 864; do
  echo "== abl$a"
  PCMS_LIB=tests/kexp/libpcms_abl$a.so timeout -k 10 120 python -u $B || exit $?
done
