#!/bin/bash
# round 6, first box: the new data-parallel bf16 / checkpointed tests and the full-size config
# tests with their parity margins recorded, then config 2 / 4 / 5 bench lines on the same box
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6a}
rm -f gpurun_out/${TAG}_margins.json
PCMS_MARGINS=gpurun_out/${TAG}_margins.json timeout -k 10 900 python -u -m pytest tests/test_dp_gpu.py tests/test_gpu_configs.py \
  -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in cfg2:"" cfg4:"--zero-fill" cfg5:"--size 256,256,96 --batch 1 --ckpt-decoder" cfg2b:""; do
  name=${cfg%%:*}; args=${cfg#*:}
  extra="--no-cpu-baseline --fp32-steps 0"
  [ "$name" = cfg2 ] && extra=""
  timeout -k 10 600 python -u bench.py $args $extra > gpurun_out/${TAG}_bench_${name}.json 2> gpurun_out/${TAG}_bench_${name}.err
  rc=$?; echo "bench $name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['config']['workload'], d['value'], d['ms_per_step'], d['clock']['sclk_mhz'], d['mfma_util_step'], d['roofline'] and (d['roofline']['frac'], d['roofline']['frac_fused']))" gpurun_out/${TAG}_bench_${name}.json
done
