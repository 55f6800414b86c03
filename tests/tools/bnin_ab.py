"""A/B of the BatchNorm + ReLU fusion into the consuming conv's staging path (test tooling;
VERDICT r3 item 4): pcms_bn_relu (y -> a in HBM) + pcms_conv3_fwd(a) against
pcms_conv3_fwd_bnin(y) on the level-0 / level-1 shapes of the DoubleConv's second conv
(models/unet3d.py:31-35).  Checks the two outputs and BatchNorm partials are bit-identical
(same bn_relu1 arithmetic, same bf16 rounding), then times each form: HIP events over 20
launches, three rotating buffer sets, median of 3 trials."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import pcms_amd  # noqa: F401
    from pcms_amd import _lib as L
    T = torch.bfloat16
    for (N, D, H, W, C) in ((2, 128, 128, 64, 64), (2, 64, 64, 32, 128)):
        nvox = N * D * H * W
        g = torch.Generator(device="cuda").manual_seed(3)
        sets = [torch.randn(nvox * C, device="cuda", generator=g).to(T) for _ in range(3)]
        sc = torch.rand(C, device="cuda", generator=g) + 0.5
        sh = torch.randn(C, device="cuda", generator=g) * 0.3
        w = torch.randn(C, C, 27, device="cuda", generator=g) * 0.05
        wp = torch.empty(L.query("pcms_conv3_pack_elems", 1, C, C), dtype=T, device="cuda")
        L.call("pcms_conv3_pack", 1, w, wp, C, C, 0)
        bias = torch.zeros(C, device="cuda")
        rows = L.query("pcms_conv3_fwd_rows", 1, N, D, H, W, C, 0, C)
        st0, st1 = torch.empty(rows * (2 * C + 1), device="cuda"), torch.empty(rows * (2 * C + 1), device="cuda")
        a = torch.empty(nvox * C, dtype=T, device="cuda")
        y0, y1 = torch.empty(nvox * C, dtype=T, device="cuda"), torch.empty(nvox * C, dtype=T, device="cuda")

        def unfused(x, y, st):
            L.call("pcms_bn_relu", 1, x, a, sc, sh, C, nvox)
            L.call("pcms_conv3_fwd", 1, a, C, None, 0, wp, bias, y, None, C, None, st, 0, N, D, H, W, C, 1)

        def fused(x, y, st):
            L.call("pcms_conv3_fwd_bnin", 1, x, C, sc, sh, wp, bias, y, st, N, D, H, W, C)

        def conv_only(x, y, st):
            L.call("pcms_conv3_fwd", 1, x, C, None, 0, wp, bias, y, None, C, None, st, 0, N, D, H, W, C, 1)

        def bn_only(x, y, st):
            L.call("pcms_bn_relu", 1, x, a, sc, sh, C, nvox)

        unfused(sets[0], y0, st0)
        fused(sets[0], y1, st1)
        torch.cuda.synchronize()
        same = torch.equal(y0.view(torch.int16), y1.view(torch.int16)) and torch.equal(st0, st1)
        res = {}
        for name, fn in (("bn_relu + conv", unfused), ("conv(bn_relu) fused", fused), ("conv alone", conv_only),
                         ("bn_relu alone", bn_only)):
            for i in range(3):
                fn(sets[i], y0, st0)
            torch.cuda.synchronize()
            tr = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(20):
                    fn(sets[i % 3], y0, st0)
                e1.record()
                e1.synchronize()
                tr.append(e0.elapsed_time(e1) / 20 * 1e3)
            res[name] = statistics.median(tr)
        print(f"{C}->{C} @ {N}x{D}x{H}x{W}: bit-identical {same}; " +
              "; ".join(f"{k} {v:.1f} us" for k, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
