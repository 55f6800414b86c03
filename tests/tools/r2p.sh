# full GPU suite, then per-launch timings of one training step
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r2p_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tests/tools/layer_times.py --out gpurun_out/r2p_layers.json > gpurun_out/r2p_layers.log 2>&1
rc2=$?; head -30 gpurun_out/r2p_layers.log; exit $rc2
