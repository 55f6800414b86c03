#!/bin/bash
# channel-major accumulators + register-direct epilogue of the 16x16x32 kernel: parity tests,
# standalone level-0 times (HEAD lib vs this tree), same-box step A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-epiT}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "fwd16 or dgrad16 or bnin or split or big" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
PCMS_LIB=$PWD/${AB:-ab/r5e}/prostate-cancer-multimodal-segmentation_amd/libpcms_hip.so timeout -k 10 120 python -u tests/tools/epi_abl.py head > gpurun_out/${TAG}_epi.txt 2>&1 || exit $?
timeout -k 10 120 python -u tests/tools/epi_abl.py chmajor >> gpurun_out/${TAG}_epi.txt 2>&1 || exit $?
grep lib gpurun_out/${TAG}_epi.txt
bash tests/tools/tree_ab.sh ${TAG} 3 ${AB:-ab/r5e} . --steps 20 --warmup 5
