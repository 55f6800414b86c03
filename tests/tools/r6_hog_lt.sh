#!/bin/bash
# per-launch times with and without one held CU (tests/kexp/cu_hog.hip), alternated
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6hl}
for r in 1 2; do
  for k in 0 1; do
    timeout -k 10 300 python -u tests/tools/layer_times.py --hog $k --out gpurun_out/${TAG}_h${k}_$r.json > gpurun_out/${TAG}_h${k}_$r.log 2>&1 || exit $?
  done
done
python - $TAG <<'PY'
import json, sys
t = sys.argv[1]
a = [json.load(open(f"gpurun_out/{t}_h0_{r}.json"))["rows"] for r in (1, 2)]
b = [json.load(open(f"gpurun_out/{t}_h1_{r}.json"))["rows"] for r in (1, 2)]
tot = [sum(x["us"] for x in rows) for rows in a + b]
print("sums h0:", tot[:2], " h1:", tot[2:])
rows = []
for i, r in enumerate(a[0]):
    u0 = min(a[0][i]["us"], a[1][i]["us"]); u1 = min(b[0][i]["us"], b[1][i]["us"])
    rows.append((u1 - u0, i, r["name"], r["desc"], u0, u1))
rows.sort(reverse=True)
for d, i, n, de, u0, u1 in rows[:40]:
    print(f"{i:4d} {n:26s} {de:36s} {u0:8.1f} -> {u1:8.1f} us  ({u1 / u0:.2f}x)")
PY
