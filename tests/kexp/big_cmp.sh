#!/bin/bash
# big-box forward: product (box depth 4, 2 WG/CU) vs depth 8 (1 WG/CU) on the level-0/1 shapes
set -o pipefail
B="tests/bench_kernels.py --only fwd,dgrad --reps 10"
echo "== product"; timeout -k 10 200 python -u $B --names conv || exit $?
echo "== bd8"; PCMS_LIB=tests/kexp/libpcms_abl1024.so timeout -k 10 200 python -u $B --names conv || exit $?
