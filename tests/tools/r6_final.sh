#!/bin/bash
# Round-end evidence on one box: the whole GPU suite (parity margins recorded), smoke, the
# default bench line, a rocprofv3 kernel-trace summary of the bench, the stem pair's HBM
# traffic (two PMC passes).  Every GPU step under its own time limit; stop at the first failure.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6z}
export PCMS_MARGINS=$PWD/gpurun_out/${TAG}_margins.jsonl
rm -f $PCMS_MARGINS
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_tests.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/${TAG}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/${TAG}_bench.json
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
R=$PWD
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${TAG}_prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/${TAG}_prof.log 2>&1)
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tests/kexp/pmc_stem_traffic.sh gpurun_out/${TAG}_stem_traffic.json
echo "pmc rc=$?"
