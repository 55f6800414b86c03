#!/bin/bash
# BN-backward apply walking the voxels from the end (BNA_REV=1 variant library libpcms_hip_rev.so,
# built by: bash tests/tools/ab_build.sh rev -DBNA_REV=1): the BN op tests on the variant, then the
# in-step layer times A/B (lib_ab.sh, rows pcms_bn_relu_bwd*).  Record: profiles/r6_bn_apply_reverse_ab.txt
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=$PWD/prostate-cancer-multimodal-segmentation_amd
PCMS_LIB=$L/libpcms_hip_rev.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_determinism.py -m gpu -k "bn or determin" -x -q --timeout 120 --timeout-method thread > gpurun_out/rev_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/rev_tests.log
[ $rc -eq 0 ] || exit $rc
bash tests/tools/lib_ab.sh libpcms_hip_rev.so bn_relu_bwd
