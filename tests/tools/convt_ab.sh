# In-step A/B of the ConvTranspose weight-gradient plan (test tooling): layer_times with the
# shape plan (A) and with pcms_convt_wgrad_taps(8) = the 8-tap plan (B), ABAB on one box.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 200 python -u tests/tools/layer_times.py --steps 5 --out gpurun_out/ctab_A$r.json > gpurun_out/ctab_A$r.log 2>&1 || exit $?
  timeout -k 10 200 python -u tests/tools/layer_times.py --steps 5 --convt-taps 8 --out gpurun_out/ctab_B$r.json > gpurun_out/ctab_B$r.log 2>&1 || exit $?
done
for v in A1 B1 A2 B2; do
  python - gpurun_out/ctab_$v.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rows = [r for r in d["rows"] if r["name"].startswith("pcms_convt_wgrad")]
print(sys.argv[1], "sum", round(sum(r["us"] for r in d["rows"])), "us; convT wgrad",
      [(r["i"], r["us"]) for r in rows], round(sum(r["us"] for r in rows), 1))
PY
done
