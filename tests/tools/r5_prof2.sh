#!/bin/bash
# deep wgrad plan A/B, then layer times + rocprofv3 kernel trace of the bench
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r5q}
timeout -k 10 300 python -u tests/tools/wgrad_deep_ab.py > gpurun_out/${TAG}_wdeep.log 2>&1 || { tail -20 gpurun_out/${TAG}_wdeep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_wdeep.log
bash tests/tools/r5_prof.sh ${TAG}
