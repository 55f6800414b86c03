"""16x16x32 big-box kernel epilogue ablation (test tooling): the product library and BG_ABL
builds (32: no bf16 slice writes, 64: no epilogue, 2: no global stores) timed on the level-0
shapes with K = 64, with the shader clock.  Usage: PCMS_LIB=<lib> python tests/tools/epi_abl.py tag"""
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # (N, D, H, W, c0, c1, Cout, cy0, stats[, bnin])
    (2, 128, 128, 64, 64, 0, 128, 64, False),   # level-0 dgrad of the decoder's first conv
    (2, 128, 128, 64, 64, 0, 64, 64, True),     # level-0 64 -> 64 forward with statistics
    (2, 128, 128, 64, 64, 64, 64, 64, True),    # level-0 decoder conv0 forward
    (2, 128, 128, 64, 64, 0, 64, 64, True, True),  # level-0 conv1 with the BN of conv0 fused in
]


def main():
    import pcms_amd  # noqa: F401
    import bench
    from pcms_amd import _lib as L
    tag = sys.argv[1] if len(sys.argv) > 1 else "product"
    probe = bench.ClockProbe()
    T = torch.bfloat16
    for (N, D, H, W, c0, c1, cout, cy0, with_stats, *bn) in SHAPES:
        bnin = bool(bn and bn[0])
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
        st = stats if with_stats else None
        isc = (torch.rand(c0, device="cuda") + 0.5) if bnin else None
        ish = torch.randn(c0, device="cuda") if bnin else None

        def run(i):
            a, b = xs[i % 2]
            L.call("pcms_conv3_fwd16", a, c0, b if c1 else None, c1, isc, ish, w16, bias, y0,
                   y1 if cy0 < cout else None, cy0, st, 0, N, D, H, W, cout)
        for rep in range(2):
            for i in range(3):
                run(i)
            torch.cuda.synchronize()
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
            print(json.dumps({"lib": tag, "shape": f"{'bn' if bnin else ''}{c0}+{c1}->{cout} {N}x{D}x{H}x{W} cy0 {cy0} stats {int(with_stats)}",
                              "us": round(us, 1), "mhz": round(mhz), "mfma_frac": round(flop / us / 1e-6 / 2.5e15, 3),
                              "mfma_frac_at_clock": round(flop / us / 1e-6 / (2.5e15 * mhz / 2400), 3)}), flush=True)


if __name__ == "__main__":
    main()
