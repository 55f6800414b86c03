#!/bin/bash
# fp32 build: the x6 weight-gradient op tests, every fp32 parity / config / determinism test,
# then the fp32 build's step rate (bench.py --precision fp32)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6f}
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py tests/test_determinism.py tests/test_gpu_configs.py \
  tests/test_gpu_blocks.py -m gpu -v --timeout 400 --timeout-method thread -k "x6 or fp32 or conv3_wgrad" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['ms_per_step'], d['clock']['sclk_mhz'])"
