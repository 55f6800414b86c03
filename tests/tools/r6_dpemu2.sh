#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6de2}
timeout -k 10 600 python -u tests/kexp/dp_emulate.py --world 8 --busbw 350 --k 16 --policies none,overlap --buckets 2,4,8,16,32,64 --rounds 2 > gpurun_out/${TAG}.txt 2>&1 || { cat gpurun_out/${TAG}.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}.txt
