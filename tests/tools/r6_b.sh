#!/bin/bash
# round 6, box b: fp32 weight-gradient box stream (tests + A/B), the CU-hog / per-launch probe,
# and a kernel trace of a short bench (where the per-step copyBuffer launches sit)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6b}
bash tests/tools/r6_x6.sh ${TAG} || exit $?
timeout -k 10 300 python -u tests/kexp/cu_hog.py 0,1,4,8,32 > gpurun_out/${TAG}_cuhog.txt 2>&1 || exit $?
cat gpurun_out/${TAG}_cuhog.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OLDPWD/gpurun_out/${TAG}_trace -o tr -- \
  python3 $OLDPWD/bench.py --steps 3 --warmup 1 --no-cpu-baseline --fp32-steps 0 > $OLDPWD/gpurun_out/${TAG}_trace.log 2>&1
echo "trace rc=$?"
