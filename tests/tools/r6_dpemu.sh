#!/bin/bash
# single-GPU emulation of the W=8 data-parallel step (tests/kexp/dp_emulate.py)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6de}
timeout -k 10 400 python -u tests/kexp/dp_emulate.py --world 8 --busbw 350 --k 16 > gpurun_out/${TAG}.txt 2>&1 || { cat gpurun_out/${TAG}.txt; exit 1; }
timeout -k 10 400 python -u tests/kexp/dp_emulate.py --world 8 --busbw 350 --k 8 --policies none,overlap >> gpurun_out/${TAG}.txt 2>&1 || exit 1
timeout -k 10 400 python -u tests/kexp/dp_emulate.py --world 8 --busbw 200 --k 16 --policies none,overlap,end >> gpurun_out/${TAG}.txt 2>&1 || exit 1
cat gpurun_out/${TAG}.txt | grep -v amdgpu.ids
