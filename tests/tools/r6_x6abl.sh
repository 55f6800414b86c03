#!/bin/bash
# fp32 build's general forward / dgrad kernel ablations (CONV_ABL builds): per-kernel time in
# the kernel trace of bench.py --precision fp32 for the product and each variant library
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6xa}; shift
export TMPDIR=/tmp
R=$PWD
for v in prod "$@"; do
  lib=""; [ "$v" != prod ] && lib=$R/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_$v.so
  rm -rf $R/gpurun_out/${TAG}_$v
  (cd /tmp && PCMS_LIB=$lib timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_$v -o run --output-format csv -- python3 $R/bench.py --precision fp32 --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 --kernel-reps 1 > $R/gpurun_out/${TAG}_$v.log 2>&1) || { echo "trace $v failed"; exit 1; }
  python3 - "$R/gpurun_out/${TAG}_$v" "$v" <<'PY'
import csv, glob, sys, collections
d, v = sys.argv[1], sys.argv[2]
rows = [r for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
agg = collections.defaultdict(float)
for r in rows:
    agg[r["Kernel_Name"].replace("(anonymous namespace)::", "")[:70]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, t in sorted(agg.items(), key=lambda x: -x[1])[:4]:
    print(f"{v:6s} {t / 4 / 1e3:8.2f} ms/step  {k}")
PY
done
