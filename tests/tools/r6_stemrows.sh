#!/bin/bash
# stem forward stats rows = workgroups: stem op tests, golden parity, then the stem / BN
# finalize kernels in the bench's kernel trace
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6sr}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py tests/test_gpu_blocks.py -m gpu -v --timeout 300 --timeout-method thread -k "stem or parity or golden or bn" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
R=$PWD
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/${TAG}_k -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --fp32-steps 0 > $R/gpurun_out/${TAG}_k.log 2>&1) || exit 1
python3 - "$R/gpurun_out/${TAG}_k" <<'PY'
import csv, glob, sys, statistics
rows = [r for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))]
for p in ("stem_fwd_direct", "colsum2", "bn_finalize_kernel", "colsum_finalize_small_kernel<false>"):
    ts = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if p in r["Kernel_Name"]]
    print(f"{p:40s} n={len(ts):4d} " + (f"median {statistics.median(ts):8.1f} us  sum/13 {sum(ts) / 13:8.1f} us" if ts else ""))
PY
