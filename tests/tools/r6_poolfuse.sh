#!/bin/bash
# MaxPool backward + BN apply fusion (engine.pool_bn_apply_fused): the whole GPU suite (its
# bit-identity test included) with it on, then the in-step ABBA A/B against the stored form and
# the layer times.  Record: profiles/r6_pool_bn_apply_fused_ab.txt
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pf_tests.log | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tests/tools/step_ab.py --rounds 8 --steps 10 --variants poolsep,poolfused > gpurun_out/pf_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; tail -2 gpurun_out/pf_ab.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tests/tools/layer_times.py --steps 3 --out gpurun_out/pf_layers.json > gpurun_out/pf_layers.log 2>&1
echo "layers rc=$?"
