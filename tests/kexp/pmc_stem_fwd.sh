#!/bin/bash
# Instruction mix and stall counters of the stem forward (test tooling): two rocprofv3 --pmc
# passes over tests/bench_stem.py fwd, CSVs under gpurun_out/pmc_stemf/
set -o pipefail
cd "$(dirname "$0")/../.."
R=$PWD
O=$R/gpurun_out/pmc_stemf
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
B="python3 $R/tests/bench_stem.py fwd 5"
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/g1 -o run --output-format csv -- $B > $O/g1.log 2>&1) || exit $?
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $O/g2 -o run --output-format csv -- $B > $O/g2.log 2>&1) || exit $?
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"{o}/g*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "stem_fwd" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
PY
