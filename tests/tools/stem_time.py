"""Stem fwd / wgrad launch times as bench.py's roofline measures them (HIP events, 3 rotating
buffer sets), without a training step around them (test tooling; PCMS_LIB picks the library)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import pcms_amd  # noqa
    from pcms_amd import _lib as L
    N, D, H, W = 2, 128, 128, 64
    nvox = N * D * H * W
    T = torch.bfloat16
    sets = [(torch.rand(nvox * 8, device="cuda").to(T), torch.empty(nvox * 64, dtype=T, device="cuda"),
             torch.randn(nvox * 64, device="cuda").to(T)) for _ in range(3)]
    w = torch.randn(64, 5, 27, device="cuda") * 0.2
    wp = torch.empty(L.query("pcms_stem_pack_elems"), dtype=T, device="cuda")
    L.call("pcms_stem_pack", w, wp, 5)
    bias = torch.randn(64, device="cuda")
    stats = torch.empty(L.query("pcms_stem_fwd_rows", N, D, H, W) * 129, device="cuda")
    bnv = [torch.rand(64, device="cuda") + 0.5 for _ in range(4)]  # scale, shift, mean, invstd
    coef = torch.randn(3 * 64, device="cuda") * 0.01
    dw = torch.zeros(64 * 5 * 27, device="cuda")
    ws = torch.empty(L.query("pcms_stem_wgrad_ws_floats", N, D, H, W, 5), device="cuda")
    fns = {"fwd": lambda s: L.call("pcms_stem_fwd", s[0], wp, bias, s[1], stats, N, D, H, W, 16),
           "fwd14": lambda s: L.call("pcms_stem_fwd", s[0], wp, bias, s[1], stats, N, D, H, W, 0),
           "wgrad": lambda s: L.call("pcms_stem_wgrad", s[0], s[2], dw, ws, 5, N, D, H, W),
           "wgrad_bn": lambda s: L.call("pcms_stem_wgrad_bn", s[0], s[2], s[1], *bnv, coef, dw, ws, 5, N, D, H, W),
           "wgrad_bn_taps": lambda s: (L.query("pcms_stem_wgrad_dense", 0),
                                       L.call("pcms_stem_wgrad_bn", s[0], s[2], s[1], *bnv, coef, dw, ws, 5, N, D, H, W),
                                       L.query("pcms_stem_wgrad_dense", 1))}
    res = {}
    for rep in range(3):
        for name, fn in fns.items():
            for i in range(3):
                fn(sets[i])
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(30):
                fn(sets[i % 3])
            e1.record()
            e1.synchronize()
            res.setdefault(name, []).append(e0.elapsed_time(e1) / 30 * 1e3)
    t = {k: min(v) for k, v in res.items()}
    print(f"fwd {t['fwd']:.1f} us (14-step {t['fwd14']:.1f})  wgrad {t['wgrad']:.1f} us  wgrad_bn {t['wgrad_bn']:.1f} us "
          f"(tap x 8-channel columns {t['wgrad_bn_taps']:.1f})  "
          f"frac(847.3 MB) {847.3e6 / ((t['fwd'] + t['wgrad_bn']) * 1e-6) / 8e12:.4f}"
          f"  (all: {res})", flush=True)


if __name__ == "__main__":
    main()
