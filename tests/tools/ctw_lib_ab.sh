# ConvTranspose weight-gradient plan timing, product vs the no-prefetch build, alternated
# (test tooling): convt_wgrad_sweep.py at TT 4 / auto, targets 512 and 1024.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=$PWD/prostate-cancer-multimodal-segmentation_amd
for v in prod nopf prod2 nopf2; do
  case $v in prod*) LIB=$L/libpcms_hip.so;; nopf*) LIB=$L/libpcms_hip_nopf.so;; esac
  PCMS_LIB=$LIB timeout -k 10 200 python -u tests/tools/convt_wgrad_sweep.py --targets 512,1024 --tts 4,0 > gpurun_out/x_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v amdgpu.ids gpurun_out/x_$v.log | grep "128->64"
done
