# Interleaved A/B of per-launch step times (test tooling): A = product library, B = the
# variant library given as $1 (file name under the package directory); ABAB order.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
B=prostate-cancer-multimodal-segmentation_amd/$1
for r in 1 2; do
  timeout -k 10 200 python -u tests/tools/layer_times.py > gpurun_out/ab_A$r.log 2>&1 || exit $?
  PCMS_LIB=$PWD/$B timeout -k 10 200 python -u tests/tools/layer_times.py > gpurun_out/ab_B$r.log 2>&1 || exit $?
done
for f in gpurun_out/ab_A1.log gpurun_out/ab_B1.log gpurun_out/ab_A2.log gpurun_out/ab_B2.log; do
  echo "== $f"; grep -E "sum of|^  pcms_(conv3_wgrad|convt_wgrad|split_epilogue|bn_relu_bwd|conv3_fwd) " $f
done
