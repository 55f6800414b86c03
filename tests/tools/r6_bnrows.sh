#!/bin/bash
# BN-backward reduce row cap 512 (product) vs 2048: BN / pool / head op tests and the GPU
# block / parity tests, the kernel-trace A/B of the BN-backward kernels, the in-step A/B
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
TAG=${1:-r6n}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_blocks.py tests/test_determinism.py -m gpu -v --timeout 300 --timeout-method thread -k "bn or pool or head or determin" > gpurun_out/${TAG}_ops.log 2>&1
rc=$?; echo "ops rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_ops.log | tail -3
[ $rc -eq 0 ] || exit $rc
bash tests/tools/r6_ktrace_ab.sh ${TAG}k rc2048 bn_relu_bwd_reduce colsum2 bn_bwd_finalize colsum_finalize_small maxpool_bwd_bn bn_relu_bwd_apply || exit 1
ROUNDS=3 bash tests/tools/r6_libab.sh ${TAG}b prod rc2048
