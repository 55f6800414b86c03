#!/bin/bash
# 16x16x32 BNIN kernel: per-piece BN apply inside the MFMA loop vs at the chunk end
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-bn16}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_step_variants.py -k "bnin" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
PCMS_LIB=$PWD/${AB}/prostate-cancer-multimodal-segmentation_amd/libpcms_hip.so timeout -k 10 150 python -u tests/tools/epi_abl.py head > gpurun_out/${TAG}_epi.txt 2>&1 || exit $?
timeout -k 10 150 python -u tests/tools/epi_abl.py inloop >> gpurun_out/${TAG}_epi.txt 2>&1 || exit $?
grep "bn64" gpurun_out/${TAG}_epi.txt
bash tests/tools/tree_ab.sh ${TAG} 3 ${AB} . --steps 20 --warmup 5
