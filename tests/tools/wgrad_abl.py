"""Weight-gradient ablation on the box (test tooling): the product kernel and WGRAD_ABL builds
(tests/tools/ab_build.sh <suf> -DWGRAD_ABL=<bits>, see conv3.hip) timed back to back on the
level-0..2 shapes of config 2, with the shader clock over the launches (bench.ClockProbe).
WGRAD_ABL_SHAPES=deep: the level-3/4 shapes instead.
Usage: python tests/tools/wgrad_abl.py [lib suffix ...]   ("" = the product library, "k32" = the
product library with pcms_conv3_wgrad_k16(0))."""
import json
import os
import statistics
import subprocess
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
PKG = os.path.join(REPO, "prostate-cancer-multimodal-segmentation_amd")

SHAPES = [  # (N, D, H, W, c0, c1, Cout)
    (2, 128, 128, 64, 64, 64, 64),
    (2, 128, 128, 64, 64, 0, 64),
    (2, 64, 64, 32, 128, 128, 128),
    (2, 32, 32, 16, 256, 0, 256),
]
if os.environ.get("WGRAD_ABL_SHAPES") == "deep":  # levels 3-4 of config 2
    SHAPES = [(2, 8, 8, 4, 1024, 0, 1024), (2, 8, 8, 4, 512, 0, 1024), (2, 16, 16, 8, 512, 0, 512),
              (2, 16, 16, 8, 512, 512, 512)]


def worker(suf):
    import pcms_amd  # noqa: F401
    import bench
    from pcms_amd import _lib as L
    probe = bench.ClockProbe()
    if suf.startswith("k32"):  # the 32x32x16 inner loop of the same library
        L.query("pcms_conv3_wgrad_k16", 0)
    res = []
    for (N, D, H, W, c0, c1, co) in SHAPES:
        nvox = N * D * H * W
        cin = c0 + c1
        T = torch.bfloat16
        x0 = torch.randn(nvox * c0, device="cuda").to(T)
        x1 = torch.randn(nvox * max(c1, 8), device="cuda").to(T)
        dy = torch.randn(nvox * co, device="cuda").to(T)
        dw = torch.zeros(co * cin * 27, device="cuda")
        ws = torch.empty(max(1, L.query("pcms_conv3_wgrad_ws_floats", 1, N, D, H, W, c0, c1, co, 256)), device="cuda")

        def run():
            L.call("pcms_conv3_wgrad", 1, x0, c0, x1 if c1 else None, c1, dy, dw, ws, N, D, H, W, co, cin, 256, 1)
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k0 = probe.stamp()
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        k1 = probe.stamp()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        mhz = statistics.median(bench.ClockProbe.mhz(k0, k1).values())
        flop = 2.0 * nvox * co * cin * 27
        res.append({"lib": suf or "product", "shape": f"{c0}+{c1}->{co} {N}x{D}x{H}x{W}", "us": round(us, 1),
                    "mhz": round(mhz), "mfma_frac": round(flop / us / 1e-6 / 2.5e15, 3),
                    "mfma_frac_at_clock": round(flop / us / 1e-6 / (2.5e15 * mhz / 2400), 3)})
    print(json.dumps(res))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--worker":
        return worker(sys.argv[2] if sys.argv[2] != "-" else "")
    sufs = [("" if a in ("product", "-") else a) for a in sys.argv[1:]] or [""]
    for rnd in range(2):
        for suf in sufs:
            env = dict(os.environ)
            if suf and not suf.startswith("k32"):
                env["PCMS_LIB"] = os.path.join(PKG, f"libpcms_hip_{suf}.so")
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--worker", suf or "-"], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                print(r.stdout, r.stderr[-3000:], flush=True)
                sys.exit(r.returncode)
            for row in json.loads(r.stdout.strip().splitlines()[-1]):
                row["round"] = rnd
                print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
