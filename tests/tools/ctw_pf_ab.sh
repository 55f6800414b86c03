# ConvTranspose weight-gradient block prefetch A/B (test tooling): op tests, the plan sweep and
# layer_times with the product library (CTW_PF=1) and libpcms_hip_nopf.so (CTW_PF=0).
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
NOPF=$PWD/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_nopf.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "convt" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pf_tests.log 2>&1 || { tail -20 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
timeout -k 10 300 python -u tests/tools/convt_wgrad_sweep.py --targets 512,1024 > gpurun_out/pf_sweep_A.log 2>&1 || exit $?
PCMS_LIB=$NOPF timeout -k 10 300 python -u tests/tools/convt_wgrad_sweep.py --targets 512,1024 > gpurun_out/pf_sweep_B.log 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u tests/tools/layer_times.py --out gpurun_out/pf_A$r.json > gpurun_out/pf_A$r.log 2>&1 || exit $?
  PCMS_LIB=$NOPF timeout -k 10 200 python -u tests/tools/layer_times.py --out gpurun_out/pf_B$r.json > gpurun_out/pf_B$r.log 2>&1 || exit $?
done
paste gpurun_out/pf_sweep_A.log gpurun_out/pf_sweep_B.log | cut -c1-200
for v in A1 B1 A2 B2; do
  python - gpurun_out/pf_$v.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rows = [r for r in d["rows"] if r["name"].startswith("pcms_convt_wgrad")]
print(sys.argv[1].split("/")[-1], "step sum", round(sum(r["us"] for r in d["rows"])), "convT wgrad", [(r["i"], r["us"]) for r in rows], round(sum(r["us"] for r in rows), 1))
PY
done
