#!/bin/bash
# BN-input apply cost in the 16x16x32 kernel: product vs BG_ABL=128 (apply skipped)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
P=prostate-cancer-multimodal-segmentation_amd
timeout -k 10 150 python -u tests/tools/epi_abl.py product > gpurun_out/bnabl.txt 2>&1 || exit $?
PCMS_LIB=$PWD/$P/libpcms_hip_b128.so timeout -k 10 150 python -u tests/tools/epi_abl.py no_bn_apply >> gpurun_out/bnabl.txt 2>&1 || exit $?
grep lib gpurun_out/bnabl.txt
