#!/bin/bash
# launch-count targets re-checked on the round-5 kernels: per-step sum of launches
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for a in "0 0" "512 0" "384 0" "0 256" "0 1024" "0 0"; do
  set -- $a
  timeout -k 10 200 python -u tests/tools/layer_times.py --wgrad-target $1 --split-target $2 > gpurun_out/tg_$1_$2.log 2>&1 || exit $?
  echo "wgrad_target $1 split_target $2: $(grep 'sum of' gpurun_out/tg_$1_$2.log) $(grep -E '^  pcms_conv3_wgrad ' gpurun_out/tg_$1_$2.log) $(grep -E '^  pcms_conv3_fwd16_split ' gpurun_out/tg_$1_$2.log)"
done
