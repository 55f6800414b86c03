#!/bin/bash
# stem forward store-offset A/B: stem op tests, standalone stem launch times (product vs the
# variant library), then the in-step A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6st}; VAR=${2:-soff0}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -v --timeout 200 --timeout-method thread -k stem > gpurun_out/${TAG}_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_ops.log | tail -3
[ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in prod $VAR; do
    lib=""; [ "$v" != prod ] && lib=$PWD/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_$v.so
    PCMS_LIB=$lib timeout -k 10 120 python -u tests/tools/stem_time.py > gpurun_out/${TAG}_t_${v}_$r.txt 2>&1 || { echo "stem_time $v failed"; exit 1; }
    echo "$v $r: $(tail -2 gpurun_out/${TAG}_t_${v}_$r.txt | tr '\n' ' ')"
  done
done
ROUNDS=3 bash tests/tools/r6_libab.sh ${TAG}b prod $VAR
