# Build an A/B variant of the product library with extra -D flags (test tooling):
#   bash tests/tools/ab_build.sh <suffix> -DFOO=1 ...  -> prostate-cancer-multimodal-segmentation_amd/libpcms_hip_<suffix>.so
set -e
cd "$(dirname "$0")/../../prostate-cancer-multimodal-segmentation_amd/csrc"
SUF=$1; shift
mkdir -p build_$SUF
for f in conv3 stem convt ops probe; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -Wno-unused-function "$@" -c $f.hip -o build_$SUF/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libpcms_hip_$SUF.so build_$SUF/*.o
rm -rf build_$SUF
