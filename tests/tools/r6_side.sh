#!/bin/bash
# deep-level conv weight gradients on the side stream: determinism + DP-shape checks at the
# chosen level, then the in-step A/B over thresholds
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6s}
timeout -k 10 900 python -u tests/tools/step_ab.py --rounds 4 --steps 10 --variants side99,side3,side2,side4 > gpurun_out/${TAG}_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -4 gpurun_out/${TAG}_ab.txt
