"""Big-box conv ablation on the box (test tooling): the product kernel and BG_ABL builds
(tests/tools/ab_build.sh <suf> -DBG_ABL=<bits>, see conv3.hip) timed back to back on the
level-0 / level-1 shapes, with the shader clock over the launches (bench.ClockProbe).
Usage: python tests/tools/big_abl.py [lib suffix ...]   ("" = the product library)."""
import json
import math
import os
import statistics
import subprocess
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
PKG = os.path.join(REPO, "prostate-cancer-multimodal-segmentation_amd")

SHAPES = [  # (N, D, H, W, c0, c1, Cout)
    (2, 128, 128, 64, 64, 0, 64),
    (2, 128, 128, 64, 64, 64, 64),
    (2, 64, 64, 32, 128, 0, 128),
]


def worker(lib_suffix):
    import pcms_amd  # noqa: F401
    import bench
    from pcms_amd import _lib as L
    k16 = lib_suffix == "k16"  # the 16x16x32 big-box kernel of the product library (pcms_conv3_fwd16)
    probe = bench.ClockProbe()
    res = []
    for (N, D, H, W, c0, c1, cout) in SHAPES:
        nvox = N * D * H * W
        cin = c0 + c1
        T = torch.bfloat16
        xs = [(torch.randn(nvox * c0, device="cuda").to(T), torch.randn(nvox * max(c1, 8), device="cuda").to(T))
              for _ in range(2)]
        y = torch.empty(nvox * cout, dtype=T, device="cuda")
        w = torch.randn(cout, cin, 27, device="cuda") / math.sqrt(27 * cin)
        wp = torch.empty(L.query("pcms_conv3_pack_elems", 1, cout, cin), dtype=T, device="cuda")
        L.call("pcms_conv3_pack", 1, w, wp, cout, cin, 0)
        bias = torch.randn(cout, device="cuda")
        stats = torch.zeros(L.query("pcms_conv3_fwd_rows", 1, N, D, H, W, c0, c1, cout) * (2 * cout + 1) + 1024,
                            device="cuda")

        if k16:
            w16 = torch.empty(L.query("pcms_conv3_pack16_elems", cout, cin), dtype=T, device="cuda")
            wd = w.reshape(-1).contiguous()
            tab = torch.tensor([[wd.data_ptr(), cout, cin, w16.data_ptr(), 0, 0, 0, 0]], dtype=torch.int64,
                               device="cuda")
            L.call("pcms_conv3_pack16", tab, 1, (cout // 32) * (cin // 32))

        def run(i):
            a, b = xs[i % 2]
            if k16:
                L.call("pcms_conv3_fwd16", a, c0, b if c1 else None, c1, None, None, w16, bias, y, None, cout, stats,
                       0, N, D, H, W, cout)
            else:
                L.call("pcms_conv3_fwd", 1, a, c0, b if c1 else None, c1, wp, bias, y, None, cout, None, stats, 0,
                       N, D, H, W, cout, 1)
        for i in range(5):
            run(i)
        torch.cuda.synchronize()
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        k0 = probe.stamp()
        e0.record()
        for i in range(reps):
            run(i)
        e1.record()
        k1 = probe.stamp()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        mhz = statistics.median(bench.ClockProbe.mhz(k0, k1).values())
        flop = 2.0 * nvox * cout * cin * 27
        res.append({"lib": lib_suffix or "product", "shape": f"{c0}+{c1}->{cout} {N}x{D}x{H}x{W}", "us": round(us, 1),
                    "mhz": round(mhz), "mfma_frac": round(flop / us / 1e-6 / 2.5e15, 3),
                    "mfma_frac_at_clock": round(flop / us / 1e-6 / (2.5e15 * mhz / 2400), 3)})
    print(json.dumps(res))


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--worker":
        return worker(sys.argv[2] if sys.argv[2] != "-" else "")
    sufs = sys.argv[1:] or [""]
    for rnd in range(2):
        for suf in sufs:
            env = dict(os.environ)
            if suf and suf != "k16":
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
