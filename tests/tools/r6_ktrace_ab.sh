#!/bin/bash
# per-kernel durations of the bench step under two libraries (rocprofv3 --kernel-trace), for
# kernels named on the command line: r6_ktrace_ab.sh TAG variant kernel-substring...
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=$1; VAR=$2; shift 2
export TMPDIR=/tmp
R=$PWD
for v in prod $VAR prod $VAR; do
  lib=""; [ "$v" != prod ] && lib=$R/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_$v.so
  rm -rf $R/gpurun_out/${TAG}_$v
  (cd /tmp && PCMS_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_$v -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --fp32-steps 0 > $R/gpurun_out/${TAG}_$v.log 2>&1) || { echo "trace $v failed"; exit 1; }
  python3 - "$R/gpurun_out/${TAG}_$v" "$v" "$@" <<'PY'
import csv, glob, sys, statistics
d, v, pats = sys.argv[1], sys.argv[2], sys.argv[3:]
rows = [r for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
for p in pats:
    ts = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if p in r["Kernel_Name"]]
    if not ts:
        print(f"{v:8s} {p:40s} n=   0")
        continue
    print(f"{v:8s} {p:40s} n={len(ts):4d} median {statistics.median(ts):8.1f} us  sum/13 {sum(ts) / 13:8.1f} us")
PY
done
