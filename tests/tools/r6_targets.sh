#!/bin/bash
# in-step A/B of the weight-gradient and split-K workgroup targets (buffers re-laid out per variant)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6t}
timeout -k 10 900 python -u tests/tools/step_ab.py --rounds 3 --steps 10 --variants ${VARIANTS:-wt256,wt192,wt320,wt384,wt512,split384,split768} > gpurun_out/${TAG}_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -8 gpurun_out/${TAG}_ab.txt
