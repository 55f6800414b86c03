#!/bin/bash
# round-5 evidence: stem HBM traffic (PMC), per-launch layer times with clocks, rocprofv3 kernel
# trace of the bench, then the default bench line
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5z}
bash tests/kexp/pmc_stem_traffic.sh gpurun_out/${TAG}_stem_traffic.json > gpurun_out/${TAG}_traffic.log 2>&1 || { tail -20 gpurun_out/${TAG}_traffic.log; exit 1; }
cat gpurun_out/${TAG}_stem_traffic.json | head -20
bash tests/tools/r5_prof.sh ${TAG} || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['clock']['sclk_mhz'], d['mfma_util_step'], d['roofline']['frac'], d['cpu_baseline'])" gpurun_out/${TAG}_bench.json
