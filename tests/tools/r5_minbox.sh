#!/bin/bash
# 16x16x32 kernel box-depth choice (pcms_conv3_big_min_boxes) re-checked: per-step sum of launches
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for m in 0 128 192 384 512 0; do
  timeout -k 10 200 python -u tests/tools/layer_times.py --big-min-boxes $m > gpurun_out/mb_$m.log 2>&1 || exit $?
  echo "big_min_boxes $m: $(grep 'sum of' gpurun_out/mb_$m.log) $(grep -E '^  pcms_conv3_fwd16 ' gpurun_out/mb_$m.log)"
done
