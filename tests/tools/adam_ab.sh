cd /root/repo && mkdir -p gpurun_out
for r in 1 2; do
  for v in prod a1 a9; do
    if [ $v = prod ]; then L=""; else L=PCMS_LIB=$PWD/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_$v.so; fi
    env $L timeout -k 10 200 python -u tests/tools/layer_times.py > gpurun_out/adam_${v}_$r.log 2>&1 || exit $?
    echo "$v $r: $(grep -E 'sum of' gpurun_out/adam_${v}_$r.log) $(grep -E '^  pcms_adam_pack_conv3 ' gpurun_out/adam_${v}_$r.log)"
  done
done
