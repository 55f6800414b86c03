# A/B of the stem kernels (test tooling): product library vs $1 (file under the package dir)
cd "$(dirname "$0")/../.."
P=prostate-cancer-multimodal-segmentation_amd
for r in 1 2; do
  for v in libpcms_hip.so $1; do
    echo -n "$v: "; PCMS_LIB=$PWD/$P/$v timeout -k 10 120 python -u tests/tools/stem_time.py 2>&1 | grep fwd | cut -c1-60 || exit 1
  done
done
