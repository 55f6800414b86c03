#!/bin/bash
# In-step A/B of variant libraries on ONE box (test tooling): bench.py (config 2, 20 steps) with
# the product library and each prostate-cancer-multimodal-segmentation_amd/libpcms_hip_<suffix>.so
# through PCMS_LIB, variants interleaved over ROUNDS rounds; prints value / ms / clock per run
# and the median per variant.  Usage: r6_libab.sh TAG suffix1 [suffix2 ...]   ("prod" = product)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=$1; shift
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    lib=""
    [ "$v" != prod ] && lib=$PWD/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_$v.so
    PCMS_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-steps 0 ${BENCH_ARGS:-} \
      > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || { echo "bench $v rc=$?"; tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
  done
done
python - "$TAG" "$ROUNDS" "$@" <<'PY'
import json, statistics, sys
tag, rounds, vs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for v in vs:
    rows = [json.load(open(f"gpurun_out/{tag}_{v}_{r}.json")) for r in range(1, rounds + 1)]
    print(f"{v:10s}", " ".join(f"{d['value']:.2f}/{d['ms_per_step']:.3f}ms@{d['clock']['sclk_mhz']}" for d in rows),
          " median ms", round(statistics.median(d["ms_per_step"] for d in rows), 3),
          " stem", [(d["roofline"]["t_fwd_us"], d["roofline"]["t_wgrad_us"]) for d in rows])
PY
