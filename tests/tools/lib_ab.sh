# Generic in-step A/B of a variant library (test tooling): layer_times with the product library
# and with prostate-cancer-multimodal-segmentation_amd/$1, ABAB; prints the rows whose name
# contains $2 and the step sums.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B=$PWD/prostate-cancer-multimodal-segmentation_amd/$1
for r in 1 2; do
  timeout -k 10 200 python -u tests/tools/layer_times.py --out gpurun_out/lab_A$r.json > gpurun_out/lab_A$r.log 2>&1 || exit $?
  PCMS_LIB=$B timeout -k 10 200 python -u tests/tools/layer_times.py --out gpurun_out/lab_B$r.json > gpurun_out/lab_B$r.log 2>&1 || exit $?
done
for v in A1 B1 A2 B2; do
  python - gpurun_out/lab_$v.json "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rows = [r for r in d["rows"] if sys.argv[2] in r["name"]]
print(sys.argv[1].split("/")[-1], "step sum", round(sum(r["us"] for r in d["rows"])), [(r["i"], r["us"]) for r in rows], round(sum(r["us"] for r in rows), 1))
PY
done
