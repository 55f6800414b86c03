cd /root/repo; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "convt" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/y_tests.log 2>&1 || { tail -20 gpurun_out/y_tests.log; exit 1; }
tail -1 gpurun_out/y_tests.log
for r in 1 2; do
  timeout -k 10 200 python -u tests/tools/layer_times.py --out gpurun_out/y_A$r.json > gpurun_out/y_A$r.log 2>&1 || exit $?
  python - gpurun_out/y_A$r.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rows = [r for r in d["rows"] if r["name"].startswith("pcms_convt_wgrad")]
print(sys.argv[1].split("/")[-1], "step sum", round(sum(r["us"] for r in d["rows"])), "convT wgrad", [(r["i"], r["us"]) for r in rows], round(sum(r["us"] for r in rows), 1))
PY
done
