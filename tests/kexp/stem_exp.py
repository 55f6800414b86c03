"""Stem kernel experiments on the box (test tooling): correctness of the candidate kernels
against the product ones, and timings.  python tests/kexp/stem_exp.py"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import pcms_amd  # noqa
    from pcms_amd import _lib as L
    ex = ctypes.CDLL(os.path.join(HERE, "libstemexp.so"))
    for n in ("exp_stem_fwd_ws", "exp_wg", "exp_read_stream", "exp_stem_fwd_v3", "exp_stem_wgrad_v2"):
        getattr(ex, n).restype = ctypes.c_int
    P = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    N, D, H, W = 2, 128, 128, 64
    nvox = N * D * H * W
    T = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    sets = []
    for i in range(3):
        x = torch.zeros(nvox, 8, device="cuda")
        x[:, :5] = torch.rand(nvox, 5, device="cuda", generator=g)
        sets.append((x.to(T).contiguous(), torch.empty(nvox * 64, dtype=T, device="cuda"),
                     torch.randn(nvox * 64, device="cuda", generator=g).to(T)))
    w = torch.randn(64, 5, 27, device="cuda", generator=g) * 0.2
    wp = torch.empty(L.query("pcms_stem_pack_elems"), dtype=T, device="cuda")
    L.call("pcms_stem_pack", w, wp, 5)
    bias = torch.randn(64, device="cuda", generator=g)
    rows = L.query("pcms_stem_fwd_rows", N, D, H, W)
    st1 = torch.zeros(rows * 129, device="cuda")
    st2 = torch.zeros(rows * 129, device="cuda")
    err = torch.zeros(4, dtype=torch.int32, device="cuda")
    # correctness: ws vs product
    x, y1, _ = sets[0]
    y2 = torch.empty_like(y1)
    L.call("pcms_stem_fwd", x, wp, bias, y1, st1, N, D, H, W, 0)
    rc = ex.exp_stem_fwd_ws(0, P(x), P(wp), P(bias), P(y2), P(st2), P(err), N, D, H, W, st())
    torch.cuda.synchronize()
    print("ws rc", rc, "err", err.tolist(), "y equal:", torch.equal(y1.view(torch.int16), y2.view(torch.int16)),
          "max|dy|", (y1.float() - y2.float()).abs().max().item(), flush=True)

    def mom(s):
        s = s.double()
        part = s[: rows * 128].view(rows, 64, 2)
        cnt = s[rows * 128: rows * 129]
        mean = part[:, :, 0].sum(0) / cnt.sum()
        nz = cnt > 0
        rm = part[nz, :, 0] / cnt[nz, None]
        m2 = part[:, :, 1].sum(0) + (cnt[nz, None] * (rm - mean) ** 2).sum(0)
        return mean, m2 / cnt.sum(), cnt.sum().item()
    m1, v1, c1 = mom(st1)
    m2, v2, c2 = mom(st2)
    print("stats counts", c1, c2, "mean rel", ((m1 - m2).abs() / v1.sqrt()).max().item(), "var rel",
          ((v1 - v2).abs() / v1).max().item(), flush=True)

    def bench(name, fn, nbytes, reps=30):
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fn(i % 3)
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e-3
        print(f"{name:48s} {t * 1e6:8.1f} us {nbytes / t / 1e9:7.0f} GB/s", flush=True)
        return t
    fb = nvox * 10 + nvox * 128
    bench("fwd product (direct)", lambda i: L.call("pcms_stem_fwd", sets[i][0], wp, bias, sets[i][1], st1, N, D, H, W, 0), fb)
    for mode, label in [(0, ""), (1, " no BN sums"), (2, " no MFMA"), (3, " no BN sums, no MFMA")]:
        bench("fwd ws (4 compute + 4 memory waves)" + label,
              lambda i, m=mode: ex.exp_stem_fwd_ws(m, P(sets[i][0]), P(wp), P(bias), P(sets[i][1]), P(st2), P(err), N, D,
                                                   H, W, st()), fb)
    print("err after timing", err.tolist(), flush=True)
    # v3: correctness vs product, then timing
    y3 = torch.empty_like(y1)
    st3 = torch.zeros(rows * 129, device="cuda")
    L.call("pcms_stem_fwd", x, wp, bias, y1, st1, N, D, H, W, 0)
    rc = ex.exp_stem_fwd_v3(0, P(x), P(wp), P(bias), P(y3), P(st3), N, D, H, W, st())
    torch.cuda.synchronize()
    m3, v3, c3 = mom(st3)
    print("v3 rc", rc, "y equal:", torch.equal(y1.view(torch.int16), y3.view(torch.int16)), "counts", c3,
          "mean rel", ((m1 - m3).abs() / v1.sqrt()).max().item(), "var rel", ((v1 - v3).abs() / v1).max().item(), flush=True)
    for rep in range(2):
        y3.fill_(7.0)
        ex.exp_stem_fwd_v3(0, P(x), P(wp), P(bias), P(y3), P(st3), N, D, H, W, st())
        torch.cuda.synchronize()
        a1 = y1.view(nvox, 64).float().cpu(); a3 = y3.view(nvox, 64).float().cpu()
        bad = (a1 != a3).nonzero()
        vox = bad[:, 0].unique()
        print("v3 rep", rep, "mismatches", bad.shape[0], "voxels", vox.numel(), "unwritten(7.0)", int((a3 == 7.0).sum()),
              "channels", bad[:, 1].unique().tolist()[:16], flush=True)
        for vv in vox[:6].tolist():
            n_, r_ = divmod(vv, D * H * W); d_, r_ = divmod(r_, H * W); h_, w_ = divmod(r_, W)
            print("   voxel", vv, "(n,d,h,w)", (n_, d_, h_, w_), "bad ch", (a1[vv] != a3[vv]).nonzero().flatten().tolist(),
                  "got", a3[vv][(a1[vv] != a3[vv])][:4].tolist(), flush=True)
    for mode, label in [(0, ""), (1, " no stores"), (2, " no MFMA"), (4, " no epilogue VALU"), (6, " no MFMA no epi"),
                        (3, " no stores no MFMA"), (14, " stores only + barrier (box geometry)"),
                        (30, " stores only, no barrier (box geometry)"), (46, " stores + barrier (contiguous)"),
                        (62, " stores only, no barrier (contiguous)"), (38, " stores + DMA + barrier (contiguous)")]:
        bench("fwd v3" + label, lambda i, m=mode: ex.exp_stem_fwd_v3(m, P(sets[i][0]), P(wp), P(bias), P(sets[i][1]),
                                                                   P(st3), N, D, H, W, st()), fb)
    dw = torch.zeros(64 * 5 * 27, device="cuda")
    ws = torch.empty(L.query("pcms_stem_wgrad_ws_floats", N, D, H, W, 5), device="cuda")
    wb = nvox * 10 + nvox * 128
    bench("wgrad product", lambda i: L.call("pcms_stem_wgrad", sets[i][0], sets[i][2], dw, ws, 5, N, D, H, W), wb)
    dw1 = torch.zeros_like(dw); dw2 = torch.zeros_like(dw)
    L.call("pcms_stem_wgrad", sets[0][0], sets[0][2], dw1, ws, 5, N, D, H, W)
    rc = ex.exp_stem_wgrad_v2(P(sets[0][0]), P(sets[0][2]), P(dw2), P(ws), 5, N, D, H, W, st())
    torch.cuda.synchronize()
    print("wgrad v2 rc", rc, "max rel diff", ((dw1 - dw2).abs().max() / dw1.abs().max()).item(), flush=True)
    bench("wgrad v2 (two-stage flush)",
          lambda i: ex.exp_stem_wgrad_v2(P(sets[i][0]), P(sets[i][2]), P(dw), P(ws), 5, N, D, H, W, st()), wb)
    part = torch.empty(1024, device="cuda")
    for mode, ns, label in [(7, 3, "compute+halo+barrier (product)"), (6, 3, "halo+barrier, no compute"),
                            (4, 3, "dy only + barrier"), (0, 3, "dy only, no barrier"), (2, 3, "halo, no barrier"),
                            (5, 3, "compute + dy + barrier"), (1, 3, "compute + dy, no barrier"),
                            (6, 2, "halo+barrier NS2"), (4, 2, "dy+barrier NS2"), (7, 2, "product NS2")]:
        nb = nvox * 128 + (nvox * 16 if mode & 2 else 0)
        bench(f"wg mode {mode} ns {ns}: {label}",
              lambda i, m=mode, n_=ns: ex.exp_wg(m, n_, P(sets[i][0]), P(sets[i][2]), P(part), N, D, H, W, st()), nb)
    for grid in (256, 1024, 4096):
        bench(f"read_stream 268MB grid {grid}",
              lambda i, gg=grid: ex.exp_read_stream(P(sets[i][2]), ctypes.c_long(nvox * 128), gg, P(part), st()),
              nvox * 128)


if __name__ == "__main__":
    main()
