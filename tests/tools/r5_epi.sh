#!/bin/bash
# epilogue ablation of the 16x16x32 kernel (libs built by tests/tools/ab_build.sh)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
P=prostate-cancer-multimodal-segmentation_amd
for v in product e32 e64 e2; do
  lib=$P/libpcms_hip_$v.so; [ $v = product ] && lib=$P/libpcms_hip.so
  PCMS_LIB=$PWD/$lib timeout -k 10 120 python -u tests/tools/epi_abl.py $v >> gpurun_out/epi_abl.txt 2>&1 || exit $?
done
cat gpurun_out/epi_abl.txt | grep lib
