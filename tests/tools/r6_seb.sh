#!/bin/bash
# Split-K epilogue with every slab load of a thread's voxels issued first (SE_BATCH=1 variant
# library libpcms_hip_seb.so, built by: bash tests/tools/ab_build.sh seb -DSE_BATCH=1): the split /
# conv op tests and the determinism tests on the variant, then the in-step layer times A/B
# (lib_ab.sh, rows pcms_split_epilogue).  Record: profiles/r6_split_epilogue_batch_ab.txt
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=$PWD/prostate-cancer-multimodal-segmentation_amd
PCMS_LIB=$L/libpcms_hip_seb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_determinism.py -m gpu -k "split or determin or conv3_fwd" -x -q --timeout 120 --timeout-method thread > gpurun_out/seb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/seb_tests.log
[ $rc -eq 0 ] || exit $rc
bash tests/tools/lib_ab.sh libpcms_hip_seb.so split_epilogue
