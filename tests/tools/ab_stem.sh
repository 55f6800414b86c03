P=prostate-cancer-multimodal-segmentation_amd
for r in 1 2; do
 for v in "" _sd4 _sd16; do
  echo -n "lib$v: "; PCMS_LIB=$PWD/$P/libpcms_hip$v.so timeout -k 10 120 python -u tests/tools/stem_time.py 2>&1 | grep fwd | cut -c1-60 || exit 1
 done
done
