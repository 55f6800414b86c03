# ConvTranspose weight-gradient variants alternated on one box (test tooling):
# convt_wgrad_sweep.py (auto plan) and layer_times with the product library, the depth-1
# prefetch build (libpcms_hip_d1.so) and the no-prefetch build (libpcms_hip_nopf.so).
# Build the variants first: tests/tools/ab_build.sh nopf -DCTW_PF=0; d1 = a library built
# from the depth-1 revision of convt.hip (git show) with the other sources.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
L=$PWD/prostate-cancer-multimodal-segmentation_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "convt" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/x_tests.log 2>&1 || { tail -20 gpurun_out/x_tests.log; exit 1; }
tail -1 gpurun_out/x_tests.log
for v in prod d1 nopf prod2 d12 nopf2; do
  case $v in prod*) LIB=$L/libpcms_hip.so;; d1*) LIB=$L/libpcms_hip_d1.so;; nopf*) LIB=$L/libpcms_hip_nopf.so;; esac
  PCMS_LIB=$LIB timeout -k 10 200 python -u tests/tools/convt_wgrad_sweep.py --targets 512 --tts 0 > gpurun_out/x_$v.log 2>&1 || exit $?
  echo "== $v $(grep -v amdgpu.ids gpurun_out/x_$v.log | awk '{print $1, $NF=="" ? "" : $(NF-6)}' | tr '\n' ' ')"
done
