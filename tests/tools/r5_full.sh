#!/bin/bash
# the whole GPU suite (timed), smoke(), then the default bench line
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5f}
t0=$(date +%s)
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "suite rc=$rc in $(( $(date +%s) - t0 )) s"
tail -12 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['clock']['sclk_mhz'], d['mfma_util_step'], d['roofline']['frac'])" gpurun_out/${TAG}_bench.json
