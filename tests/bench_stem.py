"""Time the stem kernels (fwd / wgrad) at config 2 in isolation (for rocprofv3 PMC runs).
``wgrad`` is the product's weight gradient: pcms_stem_wgrad_bn (the stem's BatchNorm-backward
apply fused in: reads dA and the pre-BN Y instead of dY)."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main():
    import pcms_amd  # noqa
    from pcms_amd import _lib as L
    which = sys.argv[1] if len(sys.argv) > 1 else "both"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    N, D, H, W = 2, 128, 128, 64
    nvox = N * D * H * W
    T = torch.bfloat16
    sets = [(torch.rand(nvox * 8, device="cuda").to(T), torch.empty(nvox * 64, dtype=T, device="cuda"),
             torch.randn(nvox * 64, device="cuda").to(T)) for _ in range(3)]
    w = torch.randn(64, 5, 27, device="cuda") * 0.2
    wp = torch.empty(L.query("pcms_stem_pack_elems"), dtype=T, device="cuda")
    L.call("pcms_stem_pack", w, wp, 5)
    bias = torch.zeros(64, device="cuda")
    stats = torch.empty(L.query("pcms_conv3_mblocks", N, D, H, W) * 129, device="cuda")
    dw = torch.zeros(64 * 5 * 27, device="cuda")
    bnv = [torch.rand(64, device="cuda") + 0.5 for _ in range(4)]  # scale, shift, mean, invstd
    coef = torch.randn(3 * 64, device="cuda") * 0.01
    ws = torch.empty(max(1, L.query("pcms_stem_wgrad_ws_floats", N, D, H, W, 5)), device="cuda")
    for name in ("fwd", "wgrad", "wgrad0", "calib"):
        # both: the product pair (fwd + fused wgrad); all: every variant and the calibrations
        if not (which == "all" or which == name or (which == "both" and name in ("fwd", "wgrad"))):
            continue
        def f(i):
            x, y, dy = sets[i % 3]
            if name == "calib":
                y.copy_(dy)          # 268 MB read + 268 MB write (torch copy kernel)
            elif name == "fwd":
                L.call("pcms_stem_fwd", x, wp, bias, y, stats, N, D, H, W, 16)  # the product: K-dense
            elif name == "wgrad0":  # the plain weight gradient over a stored dy (unfused path)
                L.call("pcms_stem_wgrad", x, dy, dw, ws, 5, N, D, H, W)
            else:
                L.call("pcms_stem_wgrad_bn", x, dy, y, *bnv, coef, dw, ws, 5, N, D, H, W)
        for i in range(3):
            f(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            f(i)
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e-3
        byts = {"fwd": nvox * 5 * 2 + nvox * 64 * 2, "wgrad": nvox * 5 * 2 + 2 * nvox * 64 * 2,
                "wgrad0": nvox * 5 * 2 + nvox * 64 * 2, "calib": 2 * nvox * 64 * 2}[name]
        print(f"stem {name}: {t * 1e6:.1f} us  {byts / t / 1e9:.0f} GB/s algorithmic", flush=True)
    if which in ("all", "calib"):
        x, y, dy = sets[0]
        for i in range(3):
            s = sets[i % 3][2].float().sum()
        torch.cuda.synchronize()
        src = [torch.empty(nvox * 64 // 2, dtype=torch.float32, device="cuda").fill_(1.0) for _ in range(3)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            s = src[i % 3].sum()
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e-3
        print(f"calib read-only sum of 268 MB: {t * 1e6:.1f} us  {nvox * 128 / t / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
