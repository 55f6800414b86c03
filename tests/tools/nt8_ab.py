"""Level-0/1 convs with 128-channel outputs on the 16x16x32 kernel: 128-channel blocks on
4-deep boxes (pcms_conv3_b16_nt8(1)) against 64-channel blocks on 8-deep boxes (0), timed back
to back with the shader clock (test tooling).  Usage: python tests/tools/nt8_ab.py"""
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # (N, D, H, W, c0, c1, Cout, cy0): fwd and dgrad shapes of levels 0-1
    (2, 128, 128, 64, 64, 0, 128, 64),      # level-0 dgrad of the decoder's first conv (split output)
    (2, 64, 64, 32, 128, 0, 128, 128),      # level-1 128 -> 128
    (2, 64, 64, 32, 64, 0, 128, 128),       # level-1 encoder conv0
    (2, 64, 64, 32, 128, 128, 128, 128),    # level-1 decoder conv0
    (2, 64, 64, 32, 128, 0, 256, 128),      # level-1 dgrad of the decoder's first conv
]


def main():
    import pcms_amd  # noqa: F401
    import bench
    from pcms_amd import _lib as L
    probe = bench.ClockProbe()
    T = torch.bfloat16
    for (N, D, H, W, c0, c1, cout, cy0) in SHAPES:
        nvox = N * D * H * W
        cin = c0 + c1
        xs = [(torch.randn(nvox * c0, device="cuda").to(T), torch.randn(nvox * max(c1, 8), device="cuda").to(T))
              for _ in range(2)]
        y0 = torch.empty(nvox * cy0, dtype=T, device="cuda")
        y1 = torch.empty(nvox * max(cout - cy0, 8), dtype=T, device="cuda")
        w = torch.randn(cout, cin, 27, device="cuda") / math.sqrt(27 * cin)
        w16 = torch.empty(L.query("pcms_conv3_pack16_elems", cout, cin), dtype=T, device="cuda")
        wd = w.reshape(-1).contiguous()
        tab = torch.tensor([[wd.data_ptr(), cout, cin, w16.data_ptr(), 0, 0, 0, 0]], dtype=torch.int64, device="cuda")
        L.call("pcms_conv3_pack16", tab, 1, (cout // 32) * (cin // 32))
        bias = torch.randn(cout, device="cuda")
        stats = torch.zeros(4096 * (2 * cout + 1) + 1024, device="cuda")
        outs = {}
        for nt8 in (1, 0, 1, 0):
            old = L.query("pcms_conv3_b16_nt8", nt8)
            st = stats if cy0 == cout else None

            def run(i):
                a, b = xs[i % 2]
                L.call("pcms_conv3_fwd16", a, c0, b if c1 else None, c1, None, None, w16, bias, y0,
                       y1 if cy0 < cout else None, cy0, st, 0, N, D, H, W, cout)
            for i in range(3):
                run(i)
            torch.cuda.synchronize()
            outs[nt8] = y0.float().clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            k0 = probe.stamp()
            e0.record()
            for i in range(20):
                run(i)
            e1.record()
            k1 = probe.stamp()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            mhz = statistics.median(bench.ClockProbe.mhz(k0, k1).values())
            flop = 2.0 * nvox * cout * cin * 27
            print(json.dumps({"nt8": nt8, "shape": f"{c0}+{c1}->{cout} {N}x{D}x{H}x{W} cy0 {cy0}", "us": round(us, 1),
                              "mhz": round(mhz), "mfma_frac": round(flop / us / 1e-6 / 2.5e15, 3),
                              "mfma_frac_at_clock": round(flop / us / 1e-6 / (2.5e15 * mhz / 2400), 3)}), flush=True)
            L.query("pcms_conv3_b16_nt8", old)
        print("max |nt8 - nt4|", (outs[1] - outs[0]).abs().max().item(), flush=True)


if __name__ == "__main__":
    main()
