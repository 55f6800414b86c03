#!/bin/bash
# Instruction mix / stall counters of the bench step's kernels (test tooling): two rocprofv3
# --pmc passes over a short bench run, summarised per kernel (mean per dispatch) for the kernel
# name substrings given: pmc_step.sh TAG substr...
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
TAG=$1; shift
O=$R/gpurun_out/pmc_$TAG
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 --kernel-reps 1 ${BENCH_ARGS:-}"
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/g1 -o run --output-format csv -- $B > $O/g1.log 2>&1) || exit $?
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $O/g2 -o run --output-format csv -- $B > $O/g2.log 2>&1) || exit $?
python3 - "$O" "$@" <<'PY'
import csv, glob, sys, collections
o, pats = sys.argv[1], sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{o}/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        for p in pats:
            if p in r["Kernel_Name"]:
                agg[p][r["Counter_Name"]].append(float(r["Counter_Value"]))
for p in pats:
    c = {k: sum(v) / len(v) for k, v in agg[p].items()}
    if not c:
        continue
    w = c.get("SQ_WAVES", 1) or 1
    wc = c.get("SQ_WAVE_CYCLES", 1) or 1
    print(f"== {p}  (dispatches {len(agg[p].get('SQ_WAVES', []))}, waves {w:.0f})")
    for k in sorted(c):
        print(f"   {k:26s} {c[k]:16.0f}  per wave {c[k] / w:12.1f}")
    print(f"   shares of wave cycles: active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}  valu {c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f}"
          f"  parked {c.get('SQ_WAIT_ANY', 0) / wc:.2f}  issue-stall {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}")
PY
