#!/bin/bash
# fp32 parity build: in-step A/B of engine / library knobs (tests/tools/step_ab.py --precision fp32)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6f32k}
timeout -k 10 1000 python -u tests/tools/step_ab.py --precision fp32 --rounds 2 --steps 4 --variants ${VARIANTS} > gpurun_out/${TAG}_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -9 gpurun_out/${TAG}_ab.txt
