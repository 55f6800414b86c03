"""Per-kernel timing (GPU) for the dominant U-Net layer shapes at config 2 (N=2, 128x128x64,
bf16): conv3 forward / dgrad / wgrad, stem, bn_relu, convT.  HIP events on the launch
stream, rotating 3 buffer sets.  Prints one line per shape with TFLOP/s and GB/s.

    python tests/bench_kernels.py [--reps 20] [--only fwd,wgrad]
"""
import argparse
import math
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def timeit(fn, reps):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fn(i % 3)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--names", default="", help="substring filter on the layer name")
    a = ap.parse_args()
    import pcms_amd  # noqa
    from pcms_amd import _lib as L
    code, T = 1, torch.bfloat16
    N = 2
    lv = [(128, 128, 64), (64, 64, 32), (32, 32, 16), (16, 16, 8), (8, 8, 4)]
    shapes = [  # (name, level, cin, cout)
        ("inc.conv3 64->64", 0, 64, 64),
        ("up4.conv0 128->64", 0, 128, 64),
        ("down1.conv3 128->128", 1, 128, 128),
        ("up3.conv0 256->128", 1, 256, 128),
        ("down2.conv3 256->256", 2, 256, 256),
        ("up2.conv0 512->256", 2, 512, 256),
        ("down3.conv3 512->512", 3, 512, 512),
        ("down4.conv3 1024->1024", 4, 1024, 1024),
    ]
    only = set(a.only.split(",")) if a.only else None
    for name, l, cin, cout in shapes:
        if a.names and a.names not in name:
            continue
        D, H, W = lv[l]
        nvox = N * D * H * W
        flop = 2.0 * nvox * cout * cin * 27
        xs = [torch.randn(nvox * cin, device="cuda").to(T) for _ in range(3)]
        ys = [torch.empty(nvox * cout, dtype=T, device="cuda") for _ in range(3)]
        dys = [torch.randn(nvox * cout, device="cuda").to(T) for _ in range(3)]
        w = torch.randn(cout, cin, 27, device="cuda") / math.sqrt(27 * cin)
        wf = torch.empty(L.query("pcms_conv3_pack_elems", code, cout, cin), dtype=T, device="cuda")
        wd = torch.empty(L.query("pcms_conv3_pack_elems", code, cin, cout), dtype=T, device="cuda")
        L.call("pcms_conv3_pack", code, w, wf, cout, cin, 0)
        L.call("pcms_conv3_pack", code, w, wd, cout, cin, 1)
        rows = L.query("pcms_conv3_mblocks", N, D, H, W)
        stats = torch.empty(rows * (cout * 2 + 1), device="cuda")
        bias = torch.zeros(cout, device="cuda")
        dw = torch.zeros(cout * cin * 27, device="cuda")
        dwt = torch.empty(L.query("pcms_conv3_wgrad_ws_floats", code, N, D, H, W, cin, 0, cout, 512), device="cuda")
        acc = torch.empty(nvox * max(cin, cout), device="cuda") if l >= 3 else None
        out = []
        if not only or "fwd" in only:
            splits = 1 if l < 3 else 4
            def f(i):
                if splits > 1:
                    L.call("pcms_conv3_fwd", code, xs[i], cin, None, 0, wf, bias, ys[i], None, cout, acc[: nvox * cout],
                           None, 0, N, D, H, W, cout, splits)
                else:
                    L.call("pcms_conv3_fwd", code, xs[i], cin, None, 0, wf, bias, ys[i], None, cout, None, stats, 0,
                           N, D, H, W, cout, 1)
            t = timeit(f, a.reps)
            out.append(f"fwd {t * 1e6:8.1f}us {flop / t / 1e12:7.1f}TF")
        if only and "fwdplain" in only:
            def f(i):
                L.call("pcms_conv3_fwd", code, xs[i], cin, None, 0, wf, None, ys[i], None, cout, None, None, 0,
                       N, D, H, W, cout, 1)
            t = timeit(f, a.reps)
            out.append(f"fwd(no bias/stats) {t * 1e6:8.1f}us {flop / t / 1e12:7.1f}TF")
        if not only or "dgrad" in only:
            splits = 1 if l < 3 else 4
            def f(i):
                if splits > 1:
                    L.call("pcms_conv3_fwd", code, dys[i], cout, None, 0, wd, None, xs[i], None, cin, acc[: nvox * cin],
                           None, 0, N, D, H, W, cin, splits)
                else:
                    L.call("pcms_conv3_fwd", code, dys[i], cout, None, 0, wd, None, xs[i], None, cin, None, None, 0,
                           N, D, H, W, cin, 1)
            t = timeit(f, a.reps)
            out.append(f"dgrad {t * 1e6:8.1f}us {flop / t / 1e12:7.1f}TF")
        if not only or "wgrad" in only:
            def f(i):
                L.call("pcms_conv3_wgrad", code, xs[i], cin, None, 0, dys[i], dw, dwt, N, D, H, W, cout, cin, 512, 1)
            t = timeit(f, a.reps)
            out.append(f"wgrad {t * 1e6:8.1f}us {flop / t / 1e12:7.1f}TF")
        print(f"{name:26s} " + " | ".join(out), flush=True)
        del xs, ys, dys
    if a.names:
        return
    # bandwidth kernels at level 0
    D, H, W = lv[0]
    nvox = N * D * H * W
    y = torch.randn(nvox * 64, device="cuda").to(T)
    aa = torch.empty_like(y)
    sc = torch.rand(64, device="cuda")
    sh = torch.randn(64, device="cuda")
    t = timeit(lambda i: L.call("pcms_bn_relu", code, y, aa, sc, sh, 64, nvox), a.reps)
    print(f"bn_relu level0           {t * 1e6:8.1f}us {2 * y.numel() * 2 / t / 1e9:7.1f}GB/s")


if __name__ == "__main__":
    main()
