cd /root/repo && mkdir -p gpurun_out
timeout -k 10 200 python -u tests/tools/layer_times.py --out gpurun_out/abl_A.json > gpurun_out/abl_A.log 2>&1 || exit $?
PCMS_LIB=$PWD/prostate-cancer-multimodal-segmentation_amd/libpcms_hip_nf.so timeout -k 10 200 python -u tests/tools/layer_times.py --out gpurun_out/abl_B.json > gpurun_out/abl_B.log 2>&1 || exit $?
python - <<'PY'
import json
A=json.load(open("gpurun_out/abl_A.json"))["rows"]; B=json.load(open("gpurun_out/abl_B.json"))["rows"]
for a,b in zip(A,B):
    if a["name"].startswith("pcms_conv3_wgrad"): print(a["i"], a["name"], a["desc"], a["us"], b["us"])
PY
