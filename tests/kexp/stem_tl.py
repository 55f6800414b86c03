"""Stem forward timeline on the box (test tooling): s_memtime stamps per wave and box from
the product kernel's STEM_STAMP hooks (tests/kexp/stem_tl.hip).  python tests/kexp/stem_tl.py"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import pcms_amd  # noqa
    from pcms_amd import _lib as L
    ex = ctypes.CDLL(os.path.join(HERE, "libstemtl.so"))
    ex.exp_stem_fwd_tl.restype = ctypes.c_int
    P = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
    N, D, H, W = 2, 128, 128, 64
    nvox = N * D * H * W
    T = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.zeros(nvox, 8, device="cuda")
    x[:, :5] = torch.rand(nvox, 5, device="cuda", generator=g)
    x = x.to(T).contiguous()
    ys = [torch.empty(nvox * 64, dtype=T, device="cuda") for _ in range(3)]
    w = torch.randn(64, 5, 27, device="cuda", generator=g) * 0.2
    wp = torch.empty(L.query("pcms_stem_pack_elems"), dtype=T, device="cuda")
    L.call("pcms_stem_pack", w, wp, 5)
    bias = torch.randn(64, device="cuda", generator=g)
    rows = L.query("pcms_stem_fwd_rows", N, D, H, W)
    st = torch.zeros(rows * 129, device="cuda")
    nb = 16
    tl = torch.zeros(256 * 8 * nb * 8, dtype=torch.int64, device="cuda")
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    y1 = torch.empty_like(ys[0])
    L.call("pcms_stem_fwd", x, wp, bias, y1, st, N, D, H, W, 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(12):
        if rep == 11:
            e0.record()
        assert ex.exp_stem_fwd_tl(P(x), P(wp), P(bias), P(ys[rep % 3]), P(st), P(tl), N, D, H, W, s) == 0
        if rep == 11:
            e1.record()
    torch.cuda.synchronize()
    print("instrumented output equal to product:", torch.equal(y1.view(torch.int16), ys[11 % 3].view(torch.int16)))
    ms = e0.elapsed_time(e1)
    a = tl.view(256, 8, nb, 8).cpu().numpy().astype(np.int64)
    t0 = a[:, :, 0, 0].min()
    tend = a[:, :, :, 5].max()
    span = tend - t0
    print(f"kernel {ms * 1e3:.1f} us; stamp span {span} ticks -> {span / (ms * 1e3):.1f} ticks/us")
    names = ["dma issue", "late epi", "mfma", "early epi", "vmcnt wait"]
    for grp, ws in (("early waves 0-3", slice(0, 4)), ("late waves 4-7", slice(4, 8))):
        b = a[:, ws]
        print(grp)
        for k in range(5):
            d = (b[:, :, :, k + 1] - b[:, :, :, k]).reshape(-1)
            print(f"   {names[k]:12s} median {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}  mean {d.mean():8.0f}")
        bw = (b[:, :, 1:, 0] - b[:, :, :-1, 5]).reshape(-1)
        print(f"   {'barrier':12s} median {np.median(bw):8.0f}  p90 {np.percentile(bw, 90):8.0f}  mean {bw.mean():8.0f}")
        per = (b[:, :, 1:, 0] - b[:, :, :-1, 0]).reshape(-1)
        print(f"   {'box period':12s} median {np.median(per):8.0f}  p90 {np.percentile(per, 90):8.0f}  mean {per.mean():8.0f}")
    first = a[:, :, 0, 0] - t0
    print("start skew across WGs: median", np.median(first), "max", first.max())
    end = a[:, :, nb - 1, 5] - t0
    print("end: median", np.median(end), "max", end.max())


if __name__ == "__main__":
    main()
