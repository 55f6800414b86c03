#!/bin/bash
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u tests/tools/big_abl.py "" walk1 sc1 stnt walk1sc1 > gpurun_out/r5_big_walk_ab.txt 2>&1 || exit $?
cat gpurun_out/r5_big_walk_ab.txt
