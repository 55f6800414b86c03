"""Level-3 convs (2 x 16x16x8, config 2): the general kernel's split-K plan (as the engine
picks it: split target 512) against the 16x16x32 split-K form (pcms_conv3_fwd16_split), each
followed by pcms_split_epilogue (bias + BN partials), timed back to back with the shader clock
(test tooling).  Usage: python tests/tools/deep3_ab.py"""
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # (N, D, H, W, c0, c1, Cout): fwd and dgrad shapes of level 3
    (2, 16, 16, 8, 256, 0, 512), (2, 16, 16, 8, 512, 0, 512), (2, 16, 16, 8, 512, 512, 512),
    (2, 16, 16, 8, 512, 0, 1024), (2, 16, 16, 8, 512, 0, 256),
]


def main():
    import pcms_amd  # noqa: F401
    import bench
    from pcms_amd import _lib as L
    probe = bench.ClockProbe()
    T = torch.bfloat16
    for (N, D, H, W, c0, c1, cout) in SHAPES:
        nvox = N * D * H * W
        cin = c0 + c1
        x0 = torch.randn(nvox * c0, device="cuda").to(T)
        x1 = torch.randn(nvox * max(c1, 8), device="cuda").to(T)
        y = torch.empty(nvox * cout, dtype=T, device="cuda")
        w = torch.randn(cout, cin, 27, device="cuda") / math.sqrt(27 * cin)
        wp = torch.empty(L.query("pcms_conv3_pack_elems", 1, cout, cin), dtype=T, device="cuda")
        L.call("pcms_conv3_pack", 1, w, wp, cout, cin, 0)
        w16 = torch.empty(L.query("pcms_conv3_pack16_elems", cout, cin), dtype=T, device="cuda")
        wd = w.reshape(-1).contiguous()
        tab = torch.tensor([[wd.data_ptr(), cout, cin, w16.data_ptr(), 0, 0, 0, 0]], dtype=torch.int64, device="cuda")
        L.call("pcms_conv3_pack16", tab, 1, (cout // 32) * (cin // 32))
        bias = torch.randn(cout, device="cuda")
        mb = L.query("pcms_conv3_mblocks", N, D, H, W)
        nch = -(-cin // L.query("pcms_conv3_chunk", 1))
        wgs = mb * (cout // 64)
        sp_g = 1 if wgs >= 192 else max(1, min(nch, -(-512 // wgs)))
        sp16 = L.query("pcms_conv3_fwd16_split_ok", N, D, H, W, c0, c1, cout)
        acc = torch.empty(max(sp_g, sp16) * nvox * cout, device="cuda")
        stats = torch.zeros(L.query("pcms_split_epilogue_rows", nvox) * (2 * cout + 1), device="cuda")
        outs = {}
        for kind in ("general", "k16", "general", "k16"):
            def run():
                if kind == "k16":
                    L.call("pcms_conv3_fwd16_split", x0, c0, x1 if c1 else None, c1, w16, acc, N, D, H, W, cout, sp16)
                    L.call("pcms_split_epilogue", 1, acc, sp16, bias, y, None, cout, stats, cout, nvox, 0)
                else:
                    L.call("pcms_conv3_fwd", 1, x0, c0, x1 if c1 else None, c1, wp, bias, y, None, cout, acc, None, 0,
                           N, D, H, W, cout, sp_g)
                    L.call("pcms_split_epilogue", 1, acc, L.query("pcms_conv3_splits", 1, cin, sp_g), bias, y, None,
                           cout, stats, cout, nvox, 0)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            outs[kind] = y.float().clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            k0 = probe.stamp()
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            k1 = probe.stamp()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            mhz = statistics.median(bench.ClockProbe.mhz(k0, k1).values())
            print(json.dumps({"kind": kind, "splits": sp16 if kind == "k16" else sp_g,
                              "shape": f"{c0}+{c1}->{cout} {N}x{D}x{H}x{W}", "us_with_epilogue": round(us, 1),
                              "mhz": round(mhz)}), flush=True)
        print("max |general - k16|", (outs["general"] - outs["k16"]).abs().max().item(), flush=True)


if __name__ == "__main__":
    main()
