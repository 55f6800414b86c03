#!/bin/bash
# ConvT weight gradient with the dout pieces staged in output-voxel order (CTW_OMAP=1 variant
# library libpcms_hip_omap.so, built by: bash tests/tools/ab_build.sh omap -DCTW_OMAP=1):
# the ConvT op tests on the variant, then the wgrad sweep at the engine's plan alternated
# product / variant, then the in-step layer times A/B.  Record: profiles/r6_convt_wgrad_omap_ab.txt
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=$PWD/prostate-cancer-multimodal-segmentation_amd
PCMS_LIB=$L/libpcms_hip_omap.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -k "convt" -x -q --timeout 120 --timeout-method thread > gpurun_out/omap_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/omap_tests.log
[ $rc -eq 0 ] || exit $rc
for v in prod omap prod2 omap2; do
  case $v in prod*) LIB=$L/libpcms_hip.so;; omap*) LIB=$L/libpcms_hip_omap.so;; esac
  PCMS_LIB=$LIB timeout -k 10 200 python -u tests/tools/convt_wgrad_sweep.py --targets 512 --tts 0 > gpurun_out/omap_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids gpurun_out/omap_$v.log
done
bash tests/tools/lib_ab.sh libpcms_hip_omap.so convt_wgrad
