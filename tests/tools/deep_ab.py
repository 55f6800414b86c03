"""Level-2 conv shapes on the general kernel (pcms_conv3_fwd, one split) against the
16x16x32 kernel on 4-deep boxes (pcms_conv3_fwd16 as the product picks it) and on 8-deep boxes
(the box-count floor lowered so they accept these grids), timed back to back with the shader
clock (test tooling, not a test).
Usage: python tests/tools/deep_ab.py"""
import json
import math
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

SHAPES = [  # (N, D, H, W, c0, c1, Cout)
    (2, 32, 32, 16, 128, 0, 256),
    (2, 32, 32, 16, 256, 0, 256),
    (2, 32, 32, 16, 256, 256, 256),
    (2, 32, 32, 16, 256, 0, 512),
]


def main():
    import pcms_amd  # noqa: F401
    import bench
    from pcms_amd import _lib as L
    probe = bench.ClockProbe()
    T = torch.bfloat16
    res = []
    for (N, D, H, W, c0, c1, cout) in SHAPES:
        nvox = N * D * H * W
        cin = c0 + c1
        xs = [(torch.randn(nvox * c0, device="cuda").to(T), torch.randn(nvox * max(c1, 8), device="cuda").to(T))
              for _ in range(2)]
        y = torch.empty(nvox * cout, dtype=T, device="cuda")
        w = torch.randn(cout, cin, 27, device="cuda") / math.sqrt(27 * cin)
        wp = torch.empty(L.query("pcms_conv3_pack_elems", 1, cout, cin), dtype=T, device="cuda")
        L.call("pcms_conv3_pack", 1, w, wp, cout, cin, 0)
        w16 = torch.empty(L.query("pcms_conv3_pack16_elems", cout, cin), dtype=T, device="cuda")
        wd = w.reshape(-1).contiguous()
        tab = torch.tensor([[wd.data_ptr(), cout, cin, w16.data_ptr(), 0, 0, 0, 0]], dtype=torch.int64, device="cuda")
        L.call("pcms_conv3_pack16", tab, 1, (cout // 32) * (cin // 32))
        bias = torch.randn(cout, device="cuda")
        stats = torch.zeros(4096 * (2 * cout + 1) + 1024, device="cuda")
        outs = {}
        for kind in ("general", "k16_4", "k16_8"):
            old = L.query("pcms_conv3_big_min_boxes", 1 if kind == "k16_8" else 256)
            def run(i):
                a, b = xs[i % 2]
                if kind != "general":
                    L.call("pcms_conv3_fwd16", a, c0, b if c1 else None, c1, None, None, w16, bias, y, None, cout,
                           stats, 0, N, D, H, W, cout)
                else:
                    L.call("pcms_conv3_fwd", 1, a, c0, b if c1 else None, c1, wp, bias, y, None, cout, None, stats,
                           0, N, D, H, W, cout, 1)
            for i in range(3):
                run(i)
            torch.cuda.synchronize()
            outs[kind] = y.float().clone()
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
            res.append({"kind": kind, "shape": f"{c0}+{c1}->{cout} {N}x{D}x{H}x{W}", "us": round(us, 1),
                        "mhz": round(mhz), "mfma_frac": round(flop / us / 1e-6 / 2.5e15, 3),
                        "mfma_frac_at_clock": round(flop / us / 1e-6 / (2.5e15 * mhz / 2400), 3)})
            print(json.dumps(res[-1]), flush=True)
            L.query("pcms_conv3_big_min_boxes", old)
        for k in ("k16_4", "k16_8"):
            d = (outs["general"] - outs[k]).abs().max().item()
            print(f"max |general - {k}|", d, "of", outs["general"].abs().max().item(), flush=True)


if __name__ == "__main__":
    main()
