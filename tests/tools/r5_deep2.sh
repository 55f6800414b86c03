#!/bin/bash
# four-deep fwd16 B prefetch distance 6 (product) vs 1 (libpcms_hip_d1.so), then the tree A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5e}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "fwd16 or dgrad16 or conv16" > gpurun_out/${TAG}_ops.log 2>&1 || { tail -30 gpurun_out/${TAG}_ops.log; exit 1; }
tail -1 gpurun_out/${TAG}_ops.log
for r in 1 2; do
  timeout -k 10 300 python -u tests/tools/deep_ab.py > gpurun_out/${TAG}_deep6_$r.log 2>&1 || { tail -20 gpurun_out/${TAG}_deep6_$r.log; exit 1; }
  PCMS_LIB=$PWD/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_d1.so timeout -k 10 300 python -u tests/tools/deep_ab.py > gpurun_out/${TAG}_deep1_$r.log 2>&1 || { tail -20 gpurun_out/${TAG}_deep1_$r.log; exit 1; }
done
grep k16_4 gpurun_out/${TAG}_deep*_*.log | grep '"us"' | cut -c1-150
bash tests/tools/tree_ab.sh ${TAG} 2 ab/r5a . || exit $?
echo done
