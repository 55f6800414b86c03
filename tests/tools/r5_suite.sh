#!/bin/bash
# GPU suite (minus the tests whose fixtures are still being generated), then the bench with
# the 16x16x32 big-box path on (default) and off (PCMS_B16=0), alternated
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5s}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "${KEXPR:-not cfg5_checkpointed_bf16_vs_reference and not config3_shape}" > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
tail -5 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-steps 0 > gpurun_out/${TAG}_b16_$r.json 2>gpurun_out/${TAG}_b16_$r.err || exit $?
  PCMS_B16=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-steps 0 > gpurun_out/${TAG}_b32_$r.json 2>gpurun_out/${TAG}_b32_$r.err || exit $?
  for v in b16 b32; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], d['clock']['sclk_mhz'], d['mfma_util_step'])" gpurun_out/${TAG}_${v}_$r.json; done
done
