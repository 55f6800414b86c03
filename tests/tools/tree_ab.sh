#!/bin/bash
# Same-box A/B of whole trees (package + library + bench.py), alternated A B A B ...:
#   tree_ab.sh TAG ROUNDS DIR_A DIR_B [bench args]
# Each DIR holds a bench.py next to its own package and built libpcms_hip.so (ab/r3, ab/r4:
# `git archive <commit> bench.py pcms_amd.py oracle include prostate-cancer-...` + make).
# "." is the working tree.  Every bench runs under its own time limit; a failure ends the script.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=$1; R=$2; A=$3; B=$4; shift 4
for r in $(seq 1 $R); do
  for side in A B; do
    d=$A; [ $side = B ] && d=$B
    timeout -k 10 240 python -u $d/bench.py --no-cpu-baseline --fp32-steps 0 "$@" \
      > gpurun_out/${TAG}_${side}$r.json 2> gpurun_out/${TAG}_${side}$r.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], (d.get('clock') or {}).get('sclk_mhz'))" \
      gpurun_out/${TAG}_${side}$r.json $side$r $d
  done
done
