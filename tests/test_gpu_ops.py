"""Kernel-level numerics on the GPU: every entry point of libpcms_hip.so against a plain
PyTorch CPU reference of the same op (fp64 on the same, already-rounded inputs).

bf16 cases feed the CPU reference the bf16-rounded inputs, so the only differences left
are fp32 accumulation order and the final bf16 rounding of the output.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _lib():
    import pcms_amd  # noqa: F401
    from pcms_amd import _lib as L
    return L


def ndhwc(x):  # (N,C,D,H,W) -> (N,D,H,W,C)
    return x.permute(0, 2, 3, 4, 1).contiguous()


def ncdhw(x):
    return x.permute(0, 4, 1, 2, 3).contiguous()


def q(x, dt):
    """round to the storage dtype (on CPU), return (cpu fp64 copy, device tensor)."""
    xd = x.to(dt)
    return xd.double(), xd.to(DEV)


def close(got, exp, tol, what=""):
    got = got.double().cpu()
    exp = exp.double().cpu()
    scale = exp.abs().max().item() + 1e-12
    err = (got - exp).abs().max().item()
    assert err <= tol * scale, f"{what}: max err {err:.3e} > {tol:.1e} * {scale:.3e}"


DTS = [(torch.float32, 0, 2e-5), (torch.bfloat16, 1, 1e-2)]
# the 3x3x3 conv entry points also take dtype 2: fp32 data, bf16x3 arithmetic (~10x the fp32
# rounding error; dtype 0 there is bf16x6, fp32-grade)
CONV_DTS = DTS + [(torch.float32, 2, 1e-4)]


def bn_moments(stats, rows, C, nvox):
    """(mean, biased var) per channel from the kernels' BN partials: [rows][C][2] rows of
    (sum, M2 about the row mean) + [rows] counts, merged in fp64 (Chan)."""
    st = stats.detach().cpu().double()
    part = st[: rows * C * 2].view(rows, C, 2)
    cnt = st[rows * C * 2: rows * C * 2 + rows]
    assert cnt.sum().item() == nvox, (cnt.sum().item(), nvox)
    mean = part[:, :, 0].sum(0) / nvox
    nz = cnt > 0
    rmean = part[nz, :, 0] / cnt[nz, None]
    m2 = part[:, :, 1].sum(0) + (cnt[nz, None] * (rmean - mean) ** 2).sum(0)
    return mean, m2 / nvox


@pytest.mark.parametrize("dt,code,tol", CONV_DTS)
@pytest.mark.parametrize("N,cin,cout,S,split", [
    (2, 8, 64, (16, 16, 16), 1),        # stem-like (5 real channels padded to 8)
    (1, 64, 64, (9, 10, 11), 1),        # odd sizes, partial boxes
    (2, 64, 128, (8, 8, 8), 1),
    (1, 128, 64, (16, 16, 16), 1),
    (2, 256, 128, (4, 4, 4), 4),        # split-K
    (1, 64, 64, (1, 1, 1), 2),          # 1-voxel volume
])
def test_conv3_fwd(dt, code, tol, N, cin, cout, S, split):
    L = _lib()
    g = torch.Generator().manual_seed(cin * 7 + cout)
    cin_real = 5 if cin == 8 else cin
    x = torch.randn(N, cin_real, *S, generator=g)
    w = torch.randn(cout, cin_real, 3, 3, 3, generator=g) / math.sqrt(27 * cin_real)
    b = torch.randn(cout, generator=g)
    xq, _ = q(x, dt)
    wq = w.to(dt).double()
    ref = F.conv3d(xq, wq, b.double(), padding=1)
    xs = torch.zeros(N, cin, *S, dtype=dt)
    xs[:, :cin_real] = x.to(dt)
    xd = ndhwc(xs).to(DEV)
    wpack = torch.empty(L.query("pcms_conv3_pack_elems", code, cout, cin_real), dtype=dt, device=DEV)
    L.call("pcms_conv3_pack", code, w.to(DEV), wpack, cout, cin_real, 0)
    y = torch.empty(N, *S, cout, dtype=dt, device=DEV)
    nvox = N * S[0] * S[1] * S[2]
    rows = L.query("pcms_conv3_fwd_rows", code, N, *S, cin, 0, cout)
    stats = torch.zeros(max(rows, L.query("pcms_split_epilogue_rows", nvox)) * (cout * 2 + 1), device=DEV)
    if split == 1:
        L.call("pcms_conv3_fwd", code, xd, cin, None, 0, wpack, b.to(DEV), y, None, cout, None, stats, 0,
               N, *S, cout, 1)
    else:
        ns = L.query("pcms_conv3_splits", code, cin, split)
        assert ns > 1
        # slabs are fully overwritten: garbage (NaN) in the workspace must not leak through
        acc = torch.full((ns * nvox * cout,), float("nan"), device=DEV)
        L.call("pcms_conv3_fwd", code, xd, cin, None, 0, wpack, b.to(DEV), y, None, cout, acc, None, 0,
               N, *S, cout, split)
        L.call("pcms_split_epilogue", code, acc, ns, b.to(DEV), y, None, cout, stats, cout, nvox, 0)
        rows = L.query("pcms_split_epilogue_rows", nvox)
        # split-K sums its slabs in a fixed order: a second run is bit-identical
        y2 = torch.empty_like(y)
        stats2 = torch.zeros_like(stats)
        L.call("pcms_conv3_fwd", code, xd, cin, None, 0, wpack, b.to(DEV), y2, None, cout, acc, None, 0,
               N, *S, cout, split)
        L.call("pcms_split_epilogue", code, acc, ns, b.to(DEV), y2, None, cout, stats2, cout, nvox, 0)
        torch.cuda.synchronize()
        assert torch.equal(y.view(torch.uint8), y2.view(torch.uint8))
        assert torch.equal(stats, stats2)
    torch.cuda.synchronize()
    close(ncdhw(y.cpu()), ref, tol, "conv3 fwd")
    mean, var = bn_moments(stats, rows, cout, nvox)
    yref = ref.transpose(0, 1).reshape(cout, -1)
    close(mean, yref.mean(1), 1e-3 if code else 1e-5, "stats mean")
    close(var, yref.var(1, unbiased=False), 1e-3 if code else 1e-5, "stats var")


@pytest.mark.parametrize("N,S,split", [(2, (1, 1, 1), 4), (2, (2, 2, 2), 1), (1, (16, 16, 16), 1),
                                       (2, (3, 5, 7), 2)])
def test_bn_stats_large_mean(N, S, split):
    """BN partial moments stay accurate when |mean| >> std (fp32 E[x^2] - E[x]^2 would lose
    most digits of the variance: BatchNorm over 2 voxels per channel at the deepest level)."""
    L = _lib()
    g = torch.Generator().manual_seed(5)
    cin, cout = 64, 64
    x = torch.randn(N, cin, *S, generator=g) * 0.05
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)
    b = 100.0 + torch.randn(cout, generator=g)
    ref = F.conv3d(x.double(), w.double(), b.double(), padding=1)
    wpack = torch.empty(L.query("pcms_conv3_pack_elems", 0, cout, cin), device=DEV)
    L.call("pcms_conv3_pack", 0, w.to(DEV), wpack, cout, cin, 0)
    y = torch.empty(N, *S, cout, device=DEV)
    nvox = N * S[0] * S[1] * S[2]
    rows = L.query("pcms_conv3_mblocks", N, *S) if split == 1 else L.query("pcms_split_epilogue_rows", nvox)
    stats = torch.zeros(rows * (cout * 2 + 1), device=DEV)
    xd = ndhwc(x).to(DEV)
    if split == 1:
        L.call("pcms_conv3_fwd", 0, xd, cin, None, 0, wpack, b.to(DEV), y, None, cout, None, stats, 0,
               N, *S, cout, 1)
    else:
        ns = L.query("pcms_conv3_splits", 0, cin, split)
        acc = torch.empty(ns * nvox * cout, device=DEV)
        L.call("pcms_conv3_fwd", 0, xd, cin, None, 0, wpack, b.to(DEV), y, None, cout, acc, None, 0,
               N, *S, cout, split)
        L.call("pcms_split_epilogue", 0, acc, ns, b.to(DEV), y, None, cout, stats, cout, nvox, 0)
    torch.cuda.synchronize()
    mean, var = bn_moments(stats, rows, cout, nvox)
    yref = ref.transpose(0, 1).reshape(cout, -1)
    # the variance of the kernel's own fp32 outputs (what BN normalises) vs the fp64 truth
    yk = ncdhw(y.cpu()).double().transpose(0, 1).reshape(cout, -1)
    vk = yk.var(1, unbiased=False)
    vr = yref.var(1, unbiased=False)
    assert ((var - vk).abs() / vk).max().item() < 1e-3
    assert ((var - vr).abs() / vr.mean()).max().item() < 2e-3
    close(mean, yref.mean(1), 1e-6, "mean")


@pytest.mark.parametrize("code", [1, 0])
def test_conv3_small_box_two_mtiles_per_wave(code):
    """Level-4 boxes (8x8x4 = 256 voxels) on four waves of 2 M-tiles: outputs bit-identical to
    two waves of 4 (the same MFMA sequence per output tile), unsplit and split-K; the BN
    partials group their sums by wave, so they agree to fp32 rounding."""
    L = _lib()
    dt = torch.bfloat16 if code == 1 else torch.float32
    g = torch.Generator().manual_seed(21)
    N, S, cin, cout = 2, (8, 8, 4), 128, 128
    x = torch.randn(N, cin, *S, generator=g).to(dt)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)
    b = torch.randn(cout, generator=g)
    wp = torch.empty(L.query("pcms_conv3_pack_elems", code, cout, cin), dtype=dt, device=DEV)
    L.call("pcms_conv3_pack", code, w.to(DEV), wp, cout, cin, 0)
    xd = ndhwc(x).to(DEV)
    nvox = N * S[0] * S[1] * S[2]
    rows = L.query("pcms_conv3_fwd_rows", code, N, *S, cin, 0, cout)
    outs = []
    old = L.query("pcms_conv3_small_box_mtw2", -1)
    try:
        for on in (1, 0):
            L.query("pcms_conv3_small_box_mtw2", on)
            y = torch.empty(N, *S, cout, dtype=dt, device=DEV)
            st = torch.zeros(rows * (cout * 2 + 1), device=DEV)
            L.call("pcms_conv3_fwd", code, xd, cin, None, 0, wp, b.to(DEV), y, None, cout, None, st, 0, N, *S, cout, 1)
            ns = L.query("pcms_conv3_splits", code, cin, 3)
            acc = torch.full((ns * nvox * cout,), float("nan"), device=DEV)
            ys = torch.empty_like(y)
            L.call("pcms_conv3_fwd", code, xd, cin, None, 0, wp, b.to(DEV), ys, None, cout, acc, None, 0, N, *S, cout, 3)
            L.call("pcms_split_epilogue", code, acc, ns, b.to(DEV), ys, None, cout, None, cout, nvox, 0)
            outs.append((y, st, ys))
    finally:
        L.query("pcms_conv3_small_box_mtw2", old)
    torch.cuda.synchronize()
    for i in (0, 2):
        assert torch.equal(outs[0][i].view(torch.uint8), outs[1][i].view(torch.uint8))
    close(outs[0][1].cpu(), outs[1][1].cpu(), 1e-5, "BN partials")
    ref = F.conv3d(x.double(), w.to(dt).double(), b.double(), padding=1)
    close(ncdhw(outs[0][0].cpu()), ref, 1e-2 if code == 1 else 2e-5, "small-box conv")


@pytest.mark.parametrize("dt,code,tol", CONV_DTS)
def test_conv3_dual_source_and_dgrad_split_output(dt, code, tol):
    """Up3D: conv over cat([skip, up]) without materialising the cat, and the dgrad whose
    output splits back into the two gradients."""
    L = _lib()
    g = torch.Generator().manual_seed(3)
    N, S, cs, cout = 2, (8, 6, 10), 64, 64
    skip = torch.randn(N, cs, *S, generator=g).to(dt)
    up = torch.randn(N, cs, *S, generator=g).to(dt)
    w = (torch.randn(cout, 2 * cs, 3, 3, 3, generator=g) / math.sqrt(27 * 2 * cs))
    ref = F.conv3d(torch.cat([skip, up], 1).double(), w.to(dt).double(), None, padding=1)
    wp = torch.empty(L.query("pcms_conv3_pack_elems", code, cout, 2 * cs), dtype=dt, device=DEV)
    L.call("pcms_conv3_pack", code, w.to(DEV), wp, cout, 2 * cs, 0)
    y = torch.empty(N, *S, cout, dtype=dt, device=DEV)
    L.call("pcms_conv3_fwd", code, ndhwc(skip).to(DEV), cs, ndhwc(up).to(DEV), cs, wp, None, y, None, cout,
           None, None, 0, N, *S, cout, 1)
    torch.cuda.synchronize()
    close(ncdhw(y.cpu()), ref, tol, "dual-source fwd")
    # dgrad: dX = conv_transpose of dy with W  (autograd reference)
    dy = torch.randn(N, cout, *S, generator=g).to(dt)
    xr = torch.cat([skip, up], 1).double().requires_grad_(True)
    F.conv3d(xr, w.to(dt).double(), None, padding=1).backward(dy.double())
    wd = torch.empty(L.query("pcms_conv3_pack_elems", code, 2 * cs, cout), dtype=dt, device=DEV)
    L.call("pcms_conv3_pack", code, w.to(DEV), wd, cout, 2 * cs, 1)
    gs = torch.empty(N, *S, cs, dtype=dt, device=DEV)
    gu = torch.empty(N, *S, cs, dtype=dt, device=DEV)
    L.call("pcms_conv3_fwd", code, ndhwc(dy).to(DEV), cout, None, 0, wd, None, gs, gu, cs, None, None, 0,
           N, *S, 2 * cs, 1)
    torch.cuda.synchronize()
    close(ncdhw(gs.cpu()), xr.grad[:, :cs], tol, "dgrad skip part")
    close(ncdhw(gu.cpu()), xr.grad[:, cs:], tol, "dgrad up part")


@pytest.mark.parametrize("N,c0,c1,cout,cy0,S,wgs", [
    (1, 64, 0, 64, 64, (8, 8, 16), 0),         # one box
    (2, 32, 32, 128, 64, (16, 8, 32), 0),      # dual source, two-pointer output, 2 channel blocks
    (1, 16, 48, 64, 64, (8, 16, 16), 0),       # chunks split unevenly between the sources
    (1, 128, 0, 192, 128, (16, 16, 16), 0),    # odd number of 64-channel blocks, split output
    (2, 64, 0, 64, 64, (16, 16, 32), 3),       # persistent: 3 slots walk 16 boxes (6, 5, 5)
    (2, 32, 32, 128, 64, (16, 16, 32), 4),     # 2 slots x 2 channel blocks, 8 boxes each
    (1, 64, 64, 64, 64, (16, 24, 16), 5),      # dual source, 5 slots over 6 boxes (2 + 1 x 4)
])
def test_conv3_fwd_big_box(N, c0, c1, cout, cy0, S, wgs):
    """Persistent big-box bf16 forward (8x8x16 boxes, 16-channel chunks, LDS-staged 16-B
    stores) vs torch conv3d on the same bf16 inputs; BN partial moments (one row per box
    slot, running merge over the slot's boxes).  The min-box threshold is lowered so these
    small grids reach it; ``wgs`` caps the grid so every workgroup walks several boxes."""
    L = _lib()
    old = L.query("pcms_conv3_big_min_boxes", 1)
    old_w = L.query("pcms_conv3_big_max_wgs", wgs)
    try:
        dt = torch.bfloat16
        g = torch.Generator().manual_seed(c0 + 5 * c1 + cout)
        x0 = torch.randn(N, c0, *S, generator=g).to(dt)
        x1 = torch.randn(N, c1, *S, generator=g).to(dt)
        cin = c0 + c1
        w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)
        b = torch.randn(cout, generator=g)
        ref = F.conv3d(torch.cat([x0, x1], 1).double(), w.to(dt).double(), b.double(), padding=1)
        wp = torch.empty(-(-cin // 32) * 27 * cout * 32, dtype=dt, device=DEV)
        L.call("pcms_conv3_pack", 1, w.to(DEV), wp, cout, cin, 0)
        y0 = torch.empty(N, *S, cy0, dtype=dt, device=DEV)
        y1 = torch.empty(N, *S, max(cout - cy0, 8), dtype=dt, device=DEV)
        nvox = N * S[0] * S[1] * S[2]
        rows = L.query("pcms_conv3_fwd_rows", 1, N, *S, c0, c1, cout)
        nbox = N * (S[0] // 8) * (S[1] // 8) * (S[2] // 16)
        assert rows == (nbox if wgs == 0 else min(nbox, wgs // (cout // 64)))  # big-box path taken
        stats = torch.zeros(rows * (cout * 2 + 1), device=DEV)
        L.call("pcms_conv3_fwd", 1, ndhwc(x0).to(DEV), c0, ndhwc(x1).to(DEV) if c1 else None, c1, wp, b.to(DEV),
               y0, y1 if cout > cy0 else None, cy0, None, stats, 0, N, *S, cout, 1)
        torch.cuda.synchronize()
        got = ncdhw(y0.cpu())
        if cout > cy0:
            got = torch.cat([got, ncdhw(y1.cpu())], 1)
        close(got, ref, 1e-2, "big-box fwd")
        mean, var = bn_moments(stats, rows, cout, nvox)
        yref = ref.transpose(0, 1).reshape(cout, -1)
        close(mean, yref.mean(1), 1e-3, "big-box stats mean")
        close(var, yref.var(1, unbiased=False), 1e-3, "big-box stats var")
    finally:
        L.query("pcms_conv3_big_min_boxes", old)
        L.query("pcms_conv3_big_max_wgs", old_w)


@pytest.mark.parametrize("dt,code,tol", CONV_DTS)
@pytest.mark.parametrize("N,c0,c1,cout,S", [
    (2, 8, 0, 64, (16, 16, 16)),
    (1, 8, 0, 64, (4, 4, 8)),           # stem channels, one box: the unsplit direct flush
    (1, 64, 0, 64, (9, 10, 11)),
    (2, 64, 64, 64, (8, 8, 8)),
    (2, 128, 0, 128, (4, 4, 4)),
    (2, 256, 0, 64, (1, 2, 1)),
    (1, 64, 64, 128, (4, 8, 8)),        # one box: the unsplit direct flush (16-B RMW of dw)
    (2, 128, 0, 128, (16, 16, 8)),      # level-3 geometry (compile-time 4x8x8 box), 16 boxes
    (2, 64, 0, 64, (8, 8, 4)),          # level-4 geometry (compile-time 8x8x4 box, 4-wide steps)
])
@pytest.mark.parametrize("store", [0, 1])
@pytest.mark.parametrize("tg", [64, 0])
def test_conv3_wgrad(dt, code, tol, N, c0, c1, cout, S, store, tg):
    """dw += (flags 0) or dw = (PCMS_GRAD_STORE: the first writer of a fresh gradient; the
    buffer's old contents must not leak through) the weight gradient.  tg: bf16 grids of at
    most tg boxes split their taps over two workgroups (tg 0: voxel splits only)."""
    L = _lib()
    old_tg = L.query("pcms_conv3_wgrad_tg_maxbox", tg)
    try:
        _wgrad_case(L, dt, code, N, c0, c1, cout, S, store)
    finally:
        L.query("pcms_conv3_wgrad_tg_maxbox", old_tg)


def _wgrad_case(L, dt, code, N, c0, c1, cout, S, store):
    g = torch.Generator().manual_seed(c0 + 3 * cout)
    cin = c0 + c1
    cin_real = 5 if cin == 8 else cin
    x = torch.zeros(N, cin, *S)
    x[:, :cin_real] = torch.randn(N, cin_real, *S, generator=g)
    x = x.to(dt)
    dy = torch.randn(N, cout, *S, generator=g).to(dt)
    xr = x[:, :cin_real].double()
    wr = torch.zeros(cout, cin_real, 3, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv3d(xr, wr, None, padding=1).backward(dy.double())
    # the stored input may carry zero pad channels (stem: 5 of 8); dw has the weight's Cin
    guard = 4096
    dw_full = torch.zeros(cout * cin_real * 27 + guard, device=DEV)
    init = torch.randn(cout * cin_real * 27, generator=g)  # dw accumulates (+=) / is overwritten
    dw_full[:-guard] = init.to(DEV)
    ws = torch.empty(L.query("pcms_conv3_wgrad_ws_floats", code, N, *S, c0, c1, cout, 256), device=DEV)
    xs = ndhwc(x).to(DEV)
    if c1:
        L.call("pcms_conv3_wgrad", code, ndhwc(x[:, :c0]).to(DEV), c0, ndhwc(x[:, c0:]).to(DEV), c1,
               ndhwc(dy).to(DEV), dw_full, ws, N, *S, cout, cin_real, 256, store)
    else:
        L.call("pcms_conv3_wgrad", code, xs, c0, None, 0, ndhwc(dy).to(DEV), dw_full, ws, N, *S, cout, cin_real,
               256, store)
    torch.cuda.synchronize()
    assert dw_full[-guard:].abs().max().item() == 0.0, "wgrad wrote past the weight gradient"
    got = (dw_full[:-guard].cpu() - (0 if store else init)).view(cout, cin_real, 3, 3, 3)
    close(got, wr.grad, 1e-4 if code else 2e-5, "wgrad")


@pytest.mark.parametrize("k16", [1, 0])
@pytest.mark.parametrize("N,c0,c1,cout,S", [
    (2, 64, 0, 64, (16, 32, 64)),      # level-0/1 geometry (box 4x4x16 or 2x8x16), voxel splits
    (1, 64, 64, 128, (8, 16, 16)),     # two sources, 2 co blocks
    (2, 128, 0, 128, (16, 16, 8)),     # compile-time 4x8x8 box
    (2, 64, 0, 64, (8, 8, 4)),         # 8x8x4 box: 4-wide rows, a step spans 8 h-rows
])
def test_conv3_wgrad_k16(k16, N, c0, c1, cout, S):
    """The compile-time-box bf16 weight gradient on v_mfma_f32_16x16x32_bf16 (the product) and
    on 32x32x16 (pcms_conv3_wgrad_k16(0)), both vs fp64, with the fresh-store and the
    accumulate flush."""
    L = _lib()
    old = L.query("pcms_conv3_wgrad_k16", k16)
    try:
        for store in (1, 0):
            _wgrad_case(L, torch.bfloat16, 1, N, c0, c1, cout, S, store)
    finally:
        L.query("pcms_conv3_wgrad_k16", old)


@pytest.mark.parametrize("x6dma", [1, 0])
@pytest.mark.parametrize("N,c0,c1,cout,S", [
    (2, 64, 64, 64, (24, 20, 40)),     # two sources, ragged edges: ~10 boxes per workgroup
    (2, 8, 0, 64, (32, 32, 32)),       # stem channels (4 taps x 8 channels per MFMA column)
    (1, 256, 0, 128, (16, 16, 8)),     # deep-level channel counts
    (2, 512, 0, 1024, (1, 1, 1)),      # level 4 of a 16^3 volume: 256 tiles, one split (direct flush)
    (2, 512, 512, 512, (2, 2, 2)),     # level 3 of a 16^3 volume, two sources
])
def test_conv3_wgrad_x6_box_stream(x6dma, N, c0, c1, cout, S):
    """fp32 build (bf16x6) weight gradient over many boxes per workgroup: the round-6 box
    stream (fp32 boxes by LDS-DMA into a staging buffer beside the previous box's MFMAs, split
    into the h / m / l tiles between boxes) and the synchronous register staging
    (pcms_conv3_wgrad_x6_dma(0)), both vs fp64 autograd at the fp32 build's bar."""
    L = _lib()
    old = L.query("pcms_conv3_wgrad_x6_dma", x6dma)
    try:
        for store in (1, 0):
            _wgrad_case(L, torch.float32, 0, N, c0, c1, cout, S, store)
    finally:
        L.query("pcms_conv3_wgrad_x6_dma", old)


@pytest.mark.parametrize("code", [1, 0])
@pytest.mark.parametrize("N,c0,c1,cout,S", [
    (2, 8, 0, 64, (16, 16, 16)),       # 1 tile: 256 split rows, 16 groups of 16
    (2, 64, 0, 64, (16, 32, 64)),      # 2 tiles: 128 rows, 8 groups
    (1, 64, 64, 128, (8, 16, 16)),     # 8 tiles: 32 rows, 2 groups
    (2, 64, 64, 64, (8, 8, 8)),        # 16 rows, one group
    (1, 256, 0, 512, (4, 4, 8)),       # deep channel counts: 2 rows
])
def test_conv3_wgrad_reduce_fused_bit_identical(code, N, c0, c1, cout, S):
    """The one-launch split-row reduction = the group-sum + reduce pair, bit for bit (fresh
    store and accumulate), and within the wgrad bar of fp64."""
    L = _lib()
    g = torch.Generator().manual_seed(5)
    dt = torch.bfloat16 if code == 1 else torch.float32
    cin = c0 + c1
    x = torch.randn(N, cin, *S, generator=g).to(dt)
    dy = torch.randn(N, cout, *S, generator=g).to(dt)
    ws = torch.empty(L.query("pcms_conv3_wgrad_ws_floats", code, N, *S, c0, c1, cout, 256), device=DEV)
    x0 = ndhwc(x[:, :c0]).to(DEV)
    x1 = ndhwc(x[:, c0:]).to(DEV) if c1 else None
    dyd = ndhwc(dy).to(DEV)
    init = torch.randn(cout * cin * 27, generator=g).to(DEV)
    old = L.query("pcms_conv3_wgrad_reduce_fused", 1)
    try:
        outs = {}
        for fused in (1, 0):
            L.query("pcms_conv3_wgrad_reduce_fused", fused)
            for store in (1, 0):
                dw = init.clone()
                L.call("pcms_conv3_wgrad", code, x0, c0, x1, c1, dyd, dw, ws, N, *S, cout, cin, 256, store)
                torch.cuda.synchronize()
                outs[fused, store] = dw.cpu()
    finally:
        L.query("pcms_conv3_wgrad_reduce_fused", old)
    for store in (1, 0):
        assert torch.equal(outs[1, store], outs[0, store]), f"store={store}"
    wr = torch.zeros(cout, cin, 3, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv3d(x.double(), wr, None, padding=1).backward(dy.double())
    close(outs[1, 1].view(cout, cin, 3, 3, 3), wr.grad, 1e-4 if code else 2e-5, "fused-reduce wgrad vs fp64")
    close((outs[1, 0] - init.cpu()).view(cout, cin, 3, 3, 3), wr.grad, 1e-4 if code else 2e-5, "accumulate")


@pytest.mark.parametrize("c0,c1,S", [(64, 0, (32, 32, 32)), (32, 32, (24, 20, 40))])
def test_conv3_wgrad_many_boxes(c0, c1, S):
    """bf16 weight gradient over a grid of many boxes (the level-0..2 voxel-split plan, partial
    last boxes, two sources) vs fp64."""
    L = _lib()
    g = torch.Generator().manual_seed(31)
    N, cout = 2, 64
    cin = c0 + c1
    x = torch.randn(N, cin, *S, generator=g).to(torch.bfloat16)
    dy = torch.randn(N, cout, *S, generator=g).to(torch.bfloat16)
    wr = torch.zeros(cout, cin, 3, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv3d(x.double(), wr, None, padding=1).backward(dy.double())
    ws = torch.empty(L.query("pcms_conv3_wgrad_ws_floats", 1, N, *S, c0, c1, cout, 256), device=DEV)
    x0 = ndhwc(x[:, :c0]).to(DEV)
    x1 = ndhwc(x[:, c0:]).to(DEV) if c1 else None
    dw = torch.full((cout * cin * 27,), float("nan"), device=DEV)
    L.call("pcms_conv3_wgrad", 1, x0, c0, x1, c1, ndhwc(dy).to(DEV), dw, ws, N, *S, cout, cin, 256, 1)
    torch.cuda.synchronize()
    close(dw.cpu().view(cout, cin, 3, 3, 3), wr.grad, 1e-4, "many-box wgrad vs fp64")


@pytest.mark.parametrize("dt,code,tol", DTS)
def test_bn_relu_fwd_bwd(dt, code, tol):
    L = _lib()
    g = torch.Generator().manual_seed(11)
    N, C, S = 2, 128, (6, 7, 8)
    nvox = N * S[0] * S[1] * S[2]
    y = (torch.randn(N, C, *S, generator=g) * 3 + 1).to(dt)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    rm, rv = torch.randn(C, generator=g), torch.rand(C, generator=g) + 0.5
    # statistics from per-voxel partial rows (one voxel per row here)
    yv = ndhwc(y).reshape(nvox, C).double()
    part = torch.cat([torch.stack([yv, torch.zeros_like(yv)], -1).flatten(), torch.ones(nvox, dtype=yv.dtype)])
    part = part.float().contiguous()
    yr = y.double().requires_grad_(True)
    rm_r, rv_r = rm.double().clone(), rv.double().clone()
    out = F.relu(F.batch_norm(yr, rm_r, rv_r, gamma.double(), beta.double(), True, 0.1, 1e-5))
    da = torch.randn(N, C, *S, generator=g).to(dt)
    out.backward(da.double())
    gd, bd = gamma.to(DEV), beta.to(DEV)
    rmd, rvd = rm.clone().to(DEV), rv.clone().to(DEV)
    nbt = torch.zeros((), dtype=torch.int64, device=DEV)
    scale, shift, mean, invstd = (torch.empty(C, device=DEV) for _ in range(4))
    ws = torch.empty(L.query("pcms_bn_ws_doubles", C), dtype=torch.float64, device=DEV)
    L.call("pcms_bn_finalize", part.to(DEV), nvox, C, float(nvox), gd, bd, rmd, rvd, nbt, 0.1, 1e-5,
           scale, shift, mean, invstd, ws)
    yd = ndhwc(y).to(DEV)
    a = torch.empty_like(yd)
    L.call("pcms_bn_relu", code, yd, a, scale, shift, C, nvox)
    rows = L.query("pcms_bn_bwd_rows", code, C, nvox)
    bpart = torch.empty(rows * C * 2, device=DEV)
    coef = torch.empty(3 * C, device=DEV)
    dgam, dbet = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dy = torch.empty_like(yd)
    L.call("pcms_bn_relu_bwd", code, ndhwc(da).to(DEV), yd, scale, shift, mean, invstd, gd, bpart, coef,
           dgam, dbet, dy, C, nvox, ws)
    torch.cuda.synchronize()
    assert int(nbt) == 1
    close(rmd.cpu(), rm_r, 1e-5, "running_mean")
    close(rvd.cpu(), rv_r, 1e-5, "running_var")
    close(ncdhw(a.cpu()), out.detach(), tol, "bn+relu fwd")
    close(ncdhw(dy.cpu()), yr.grad, 5 * tol, "bn+relu bwd")
    # reference grads of gamma/beta through autograd
    gr = gamma.double().requires_grad_(True)
    br = beta.double().requires_grad_(True)
    F.relu(F.batch_norm(y.double(), None, None, gr, br, True, 0.1, 1e-5)).backward(da.double())
    close(dgam.cpu(), gr.grad, 1e-3 if code else 1e-5, "dgamma")
    close(dbet.cpu(), br.grad, 1e-3 if code else 1e-5, "dbeta")


@pytest.mark.parametrize("dt,code,tol", DTS)
def test_maxpool_fwd_bwd(dt, code, tol):
    L = _lib()
    g = torch.Generator().manual_seed(5)
    N, C, S = 2, 64, (7, 6, 9)
    a = torch.randn(N, C, *S, generator=g)
    a[:, :, :2, :2, :2] = 0.0  # ties among zeros (ReLU outputs)
    a = a.to(dt)
    ar = a.double().requires_grad_(True)
    p = F.max_pool3d(ar, 2)
    dp = torch.randn(p.shape, generator=g).to(dt)
    p.backward(dp.double())
    ad = ndhwc(a).to(DEV)
    pd = torch.empty(N, S[0] // 2, S[1] // 2, S[2] // 2, C, dtype=dt, device=DEV)
    L.call("pcms_maxpool_fwd", code, ad, pd, N, *S, C)
    base = torch.randn(N, C, *S, generator=g).to(dt)
    da = ndhwc(base).to(DEV)
    L.call("pcms_maxpool_bwd", code, ad, ndhwc(dp).to(DEV), da, N, *S, C)
    torch.cuda.synchronize()
    close(ncdhw(pd.cpu()), p.detach(), 0, "maxpool fwd")
    close(ncdhw(da.cpu()), base.double() + ar.grad, tol, "maxpool bwd (accumulate)")


@pytest.mark.parametrize("dt,code,tol", DTS)
@pytest.mark.parametrize("S,C", [((8, 6, 10), 64), ((7, 5, 9), 128), ((3, 4, 5), 512)])
def test_bn_relu_pool_and_maxpool_bwd_bn(dt, code, tol, S, C):
    """Down3D boundary fusion vs the unfused passes on the same inputs, odd (floor-mode)
    sizes included: pcms_bn_relu_pool == pcms_bn_relu + pcms_maxpool_fwd bit for bit;
    pcms_maxpool_bwd_bn leaves the same da as pcms_maxpool_bwd (bit for bit) and its BN
    partial rows, finished by pcms_bn_relu_bwd_finish, give pcms_bn_relu_bwd's dy / dgamma /
    dbeta up to summation order; and the whole chain against fp64 autograd of
    maxpool(relu(batch_norm(y)))."""
    L = _lib()
    g = torch.Generator().manual_seed(6)
    N = 2
    nvox = N * S[0] * S[1] * S[2]
    y = (torch.randn(N, C, *S, generator=g) * 1.5).to(dt)
    y[:, :, :2, :2, :2] = -3.0  # ReLU ties at zero inside a pooling cell
    y = y.to(dt)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    P = tuple(s // 2 for s in S)
    dp = torch.randn(N, C, *P, generator=g).to(dt)
    skip = torch.randn(N, C, *S, generator=g).to(dt)   # the skip-path part of the output gradient
    yr = y.double().requires_grad_(True)
    gr, brr = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    a_ref = F.relu(F.batch_norm(yr, None, None, gr, brr, True, 0.1, 1e-5))
    p_ref = F.max_pool3d(a_ref, 2)
    torch.autograd.backward([p_ref, a_ref], [dp.double(), skip.double()])
    m = y.double().mean((0, 2, 3, 4))
    inv = 1.0 / torch.sqrt(y.double().var((0, 2, 3, 4), unbiased=False) + 1e-5)
    sc = (gamma.double() * inv).float().to(DEV)
    sh = (beta.double() - m * gamma.double() * inv).float().to(DEV)
    mean, invstd, gd = m.float().to(DEV), inv.float().to(DEV), gamma.to(DEV)
    yd, dpd = ndhwc(y).to(DEV), ndhwc(dp).to(DEV)
    # forward
    a0, p0 = torch.empty_like(yd), torch.empty(N, *P, C, dtype=dt, device=DEV)
    L.call("pcms_bn_relu", code, yd, a0, sc, sh, C, nvox)
    L.call("pcms_maxpool_fwd", code, a0, p0, N, *S, C)
    a1, p1 = torch.full_like(a0, float("nan")), torch.full_like(p0, float("nan"))
    L.call("pcms_bn_relu_pool", code, yd, a1, p1, sc, sh, N, *S, C)
    # backward
    rows = max(L.query("pcms_bn_bwd_rows", code, C, nvox), L.query("pcms_maxpool_bwd_bn_rows", code, N, *S, C))
    part = torch.empty(rows * C * 2, device=DEV)
    coef = torch.empty(3 * C, device=DEV)
    bnws = torch.empty(L.query("pcms_bn_ws_doubles", C), dtype=torch.float64, device=DEV)
    da0 = ndhwc(skip).to(DEV)
    L.call("pcms_maxpool_bwd", code, a0, dpd, da0, N, *S, C)
    dg0, db0, dy0 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV), torch.empty_like(yd)
    L.call("pcms_bn_relu_bwd", code, da0, yd, sc, sh, mean, invstd, gd, part, coef, dg0, db0, dy0, C, nvox, bnws)
    da1 = ndhwc(skip).to(DEV)
    L.call("pcms_maxpool_bwd_bn", code, yd, sc, sh, mean, invstd, dpd, da1, part, N, *S, C)
    r1 = L.query("pcms_maxpool_bwd_bn_rows", code, N, *S, C)
    dg1, db1, dy1 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV), torch.full_like(yd, float("nan"))
    L.call("pcms_bn_relu_bwd_finish", code, da1, yd, sc, sh, mean, invstd, gd, part, r1, coef, dg1, db1, dy1, C, nvox,
           bnws)
    part1 = part[: r1 * C * 2].clone()
    # the consumer form (engine.pool_bn_apply_fused): the same rows without rewriting da, then
    # the pooled part added again inside the apply -- the same dy bits
    da2 = ndhwc(skip).to(DEV)
    part.fill_(float("nan"))
    L.call("pcms_maxpool_bwd_bn_sums", code, yd, sc, sh, mean, invstd, dpd, da2, part, N, *S, C)
    part2 = part[: r1 * C * 2].clone()
    dg2, db2, dy2 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV), torch.full_like(yd, float("nan"))
    L.call("pcms_bn_relu_bwd_finish", code, da2, yd, sc, sh, mean, invstd, gd, part, r1, coef, dg2, db2, None, C, nvox,
           bnws)
    L.call("pcms_maxpool_bn_apply", code, yd, sc, sh, mean, invstd, coef, dpd, da2, dy2, N, *S, C)
    torch.cuda.synchronize()
    assert torch.equal(da2, ndhwc(skip).to(DEV)), "pcms_maxpool_bwd_bn_sums wrote da"
    assert torch.equal(part1, part2), "partial rows differ"
    assert torch.equal(dg1, dg2) and torch.equal(db1, db2)
    bad = (dy1 != dy2).nonzero()
    assert bad.numel() == 0, (bad[:8].tolist(), dy1[dy1 != dy2][:8].tolist(), dy2[dy1 != dy2][:8].tolist())
    assert torch.equal(a0, a1) and torch.equal(p0, p1)
    assert torch.equal(da0, da1)
    close(dg1.cpu(), dg0.cpu(), 1e-5, "dgamma fused vs unfused")
    close(db1.cpu(), db0.cpu(), 1e-5, "dbeta fused vs unfused")
    close(ncdhw(dy1.cpu()), ncdhw(dy0.cpu()), 1e-5 if not code else 1e-2, "dy fused vs unfused")
    close(ncdhw(p1.cpu()), p_ref.detach(), 1e-5 if not code else 1e-2, "pool vs fp64")
    if code == 0:  # bf16: rounding makes ties among a cell's outputs, so the argmax (and with
        # it where dp lands) legitimately differs from the fp64 run; the fused == unfused checks
        # above are the bf16 bar
        close(ncdhw(dy1.cpu()), yr.grad, 1e-4, "dy vs fp64")
        close(dg1.cpu(), gr.grad, 1e-4, "dgamma vs fp64")
        close(db1.cpu(), brr.grad, 1e-4, "dbeta vs fp64")


@pytest.mark.parametrize("dt,code,tol", DTS)
@pytest.mark.parametrize("Sin,Sout,cin,cout",[((4, 4, 2), (8, 8, 4), 128, 64), ((2, 2, 3), (5, 4, 7), 128, 64),
                                               ((8, 8, 6), (16, 16, 12), 256, 128),  # > 1 tile, 2 co chunks
                                               ((8, 8, 4), (16, 16, 8), 1024, 512),  # level 4 (split dgrad)
                                               ((31, 32, 17), (62, 64, 34), 128, 64)])  # fp32: 4 M-tiles per wave, ragged
def test_convt(dt, code, tol, Sin, Sout, cin, cout):
    L = _lib()
    g = torch.Generator().manual_seed(9)
    N = 2
    x = torch.randn(N, cin, *Sin, generator=g).to(dt)
    w = (torch.randn(cin, cout, 2, 2, 2, generator=g) / math.sqrt(cin)).to(dt)
    b = torch.randn(cout, generator=g)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    u = F.conv_transpose3d(xr, wr, br, stride=2)
    dz, dyy, dxx = (Sout[i] - u.shape[2 + i] for i in range(3))
    up = F.pad(u, [dxx // 2, dxx - dxx // 2, dyy // 2, dyy - dyy // 2, dz // 2, dz - dz // 2])
    gout = torch.randn(up.shape, generator=g).to(dt)
    up.backward(gout.double())
    fp = torch.empty(L.query("pcms_convt_pack_elems", code, cin, cout), dtype=dt, device=DEV)
    dp = torch.empty(L.query("pcms_convt_pack_elems", code, cin, cout), dtype=dt, device=DEV)
    wdev = w.float().to(DEV)
    L.call("pcms_convt_pack", code, wdev, fp, cin, cout, 0)
    L.call("pcms_convt_pack", code, wdev, dp, cin, cout, 1)
    out = torch.full((N, *Sout, cout), float("nan"), dtype=dt, device=DEV)
    L.call("pcms_convt_fwd", code, ndhwc(x).to(DEV), fp, b.to(DEV), out, N, *Sin, cin, cout, *Sout)
    # K-split forward (fp32 slabs summed in a fixed order with the bias) where the grid is small
    nfs = L.query("pcms_convt_fwd_ws_floats", N, *Sin, cin, cout)
    outs = torch.full_like(out, float("nan"))
    fws = torch.full((max(nfs, 1),), float("nan"), device=DEV)
    L.call("pcms_convt_fwd_ws", code, ndhwc(x).to(DEV), fp, b.to(DEV), outs, fws, N, *Sin, cin, cout, *Sout)
    god = ndhwc(gout).to(DEV)
    dx = torch.empty(N, *Sin, cin, dtype=dt, device=DEV)
    L.call("pcms_convt_dgrad", code, god, dp, dx, N, *Sin, cin, cout, *Sout)
    # K-split dgrad (fp32 slabs in ws, summed in a fixed order) where the grid is small
    nws = L.query("pcms_convt_dgrad_ws_floats", N, *Sin, cin, cout)
    assert nws > 0 or cin % 128, "small grids split the dgrad"
    dxs = torch.full_like(dx, float("nan"))
    dws = torch.full((max(nws, 1),), float("nan"), device=DEV)
    L.call("pcms_convt_dgrad_ws", code, god, dp, dxs, dws, N, *Sin, cin, cout, *Sout)
    dw = torch.zeros(cin, cout, 2, 2, 2, device=DEV)
    ws = torch.empty(L.query("pcms_convt_wgrad_ws_floats", N, *Sin, cin, cout, 64), device=DEV)
    L.call("pcms_convt_wgrad", code, ndhwc(x).to(DEV), god, dw, ws, N, *Sin, cin, cout, *Sout, 64)
    db = torch.zeros(cout, device=DEV)
    bws = torch.empty(L.query("pcms_box_channel_sum_ws_floats", code, N, cout, 2 * Sin[0], 2 * Sin[1], 2 * Sin[2]),
                      device=DEV)
    L.call("pcms_box_channel_sum", code, god, db, bws, N, *Sout, cout, dz // 2, dyy // 2, dxx // 2,
           2 * Sin[0], 2 * Sin[1], 2 * Sin[2])
    # weight and bias gradients in one call (the bias from the weight gradient's own read of
    # dout on the bf16 128-ci path, else the box sum after it)
    dw2, db2 = torch.zeros_like(dw), torch.zeros_like(db)
    bws2 = torch.empty(L.query("pcms_convt_wgrad_bias_ws_floats", code, N, *Sin, cin, cout, 64), device=DEV)
    L.call("pcms_convt_wgrad_bias", code, ndhwc(x).to(DEV), god, dw2, db2, ws, bws2, N, *Sin, cin, cout, *Sout, 64)
    torch.cuda.synchronize()
    close(ncdhw(out.cpu()), up.detach(), tol, "convT fwd (+pad)")
    close(ncdhw(outs.cpu()), up.detach(), tol, "convT fwd (+pad, K-split)")
    assert nfs > 0 or not code or (Sin, cin) not in (((8, 8, 4), 1024), ((2, 2, 3), 128)), "small grids split"
    close(ncdhw(dx.cpu()), xr.grad, tol, "convT dgrad")
    close(ncdhw(dxs.cpu()), xr.grad, tol, "convT dgrad (K-split)")
    close(dw.cpu(), wr.grad, 1e-4 if code else 2e-5, "convT wgrad")
    close(db.cpu(), br.grad, 1e-4 if code else 1e-5, "convT bias grad")
    assert torch.equal(dw2, dw), "fused wgrad + bias: the same weight gradient"
    close(db2.cpu(), br.grad, 1e-4 if code else 1e-5, "convT bias grad (fused)")


@pytest.mark.parametrize("tt", [0, 8, 4, 2])
@pytest.mark.parametrize("Sin,Sout,cin,cout,target", [((8, 8, 4), (16, 16, 8), 1024, 512, 256),   # one split: dw direct
                                                      ((8, 8, 4), (16, 16, 8), 1024, 512, 1024),
                                                      ((5, 6, 3), (11, 12, 7), 256, 128, 2048),  # ragged, F.pad ring
                                                      ((16, 16, 8), (32, 32, 16), 512, 256, 1024),
                                                      ((2, 2, 3), (5, 4, 7), 128, 64, 512)])  # one block: direct, every TT
def test_convt_wgrad_taps(tt, Sin, Sout, cin, cout, target):
    """The bf16 ConvTranspose weight + bias gradient with the 8 taps over 8 / TT workgroups
    (fewer voxel splits; one split writes dw directly, += onto what it holds) against fp64."""
    L = _lib()
    g = torch.Generator().manual_seed(11)
    N = 2
    x = torch.randn(N, cin, *Sin, generator=g).bfloat16()
    w = (torch.randn(cin, cout, 2, 2, 2, generator=g) / math.sqrt(cin)).bfloat16()
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = torch.zeros(cout, dtype=torch.float64, requires_grad=True)
    u = F.conv_transpose3d(xr, wr, br, stride=2)
    dz, dyy, dxx = (Sout[i] - u.shape[2 + i] for i in range(3))
    up = F.pad(u, [dxx // 2, dxx - dxx // 2, dyy // 2, dyy - dyy // 2, dz // 2, dz - dz // 2])
    gout = torch.randn(up.shape, generator=g).bfloat16()
    up.backward(gout.double())
    w0 = torch.randn(cin, cout, 2, 2, 2, generator=g)  # the accumulation target's prior content
    b0 = torch.randn(cout, generator=g)
    old = L.query("pcms_convt_wgrad_taps", tt)
    try:
        ws = torch.empty(L.query("pcms_convt_wgrad_ws_floats", N, *Sin, cin, cout, target), device=DEV)
        bws = torch.empty(L.query("pcms_convt_wgrad_bias_ws_floats", 1, N, *Sin, cin, cout, target), device=DEV)
        dw, db = w0.to(DEV), b0.to(DEV)
        L.call("pcms_convt_wgrad_bias", 1, ndhwc(x).to(DEV), ndhwc(gout).to(DEV), dw, db, ws, bws, N, *Sin, cin,
               cout, *Sout, target)
        torch.cuda.synchronize()
    finally:
        L.query("pcms_convt_wgrad_taps", old)
    close(dw.cpu() - w0, wr.grad, 1e-4, f"convT wgrad TT={tt}")
    close(db.cpu() - b0, br.grad, 1e-4, f"convT bias grad TT={tt}")


@pytest.mark.parametrize("code", [1, 0])
@pytest.mark.parametrize("Sin,Sout,cin,cout,target", [((16, 16, 8), (32, 32, 16), 512, 256, 1024),
                                                      ((32, 32, 16), (64, 64, 32), 128, 64, 512),   # > 16 splits
                                                      ((5, 6, 3), (11, 12, 7), 256, 128, 2048),
                                                      ((8, 8, 4), (16, 16, 8), 1024, 512, 256)])    # direct
def test_convt_reduce_fused_bit_identical(code, Sin, Sout, cin, cout, target):
    """The ConvTranspose weight + bias gradient with its split rows and bias rows summed by one
    launch = the group-sum / reduce / bias-reduce launches, bit for bit (+= onto prior dw, db)."""
    L = _lib()
    g = torch.Generator().manual_seed(12)
    N = 2
    dt = torch.bfloat16 if code == 1 else torch.float32
    x = ndhwc(torch.randn(N, cin, *Sin, generator=g).to(dt)).to(DEV)
    gout = ndhwc(torch.randn(N, cout, *Sout, generator=g).to(dt)).to(DEV)
    w0 = torch.randn(cin * cout * 8, generator=g).to(DEV)
    b0 = torch.randn(cout, generator=g).to(DEV)
    ws = torch.empty(L.query("pcms_convt_wgrad_ws_floats", N, *Sin, cin, cout, target), device=DEV)
    bws = torch.empty(max(1, L.query("pcms_convt_wgrad_bias_ws_floats", code, N, *Sin, cin, cout, target)), device=DEV)
    old = L.query("pcms_convt_reduce_fused", 1)
    outs = {}
    try:
        for fused in (1, 0):
            L.query("pcms_convt_reduce_fused", fused)
            dw, db = w0.clone(), b0.clone()
            L.call("pcms_convt_wgrad_bias", code, x, gout, dw, db, ws, bws, N, *Sin, cin, cout, *Sout, target)
            torch.cuda.synchronize()
            outs[fused] = (dw.cpu(), db.cpu())
    finally:
        L.query("pcms_convt_reduce_fused", old)
    assert torch.equal(outs[1][0], outs[0][0]), "dw"
    assert torch.equal(outs[1][1], outs[0][1]), "db"


@pytest.mark.parametrize("Sin,Sout", [((32, 32, 24), (64, 64, 48)), ((24, 20, 12), (49, 41, 25))])
def test_convt_fwd_stream(Sin, Sout):
    """The persistent level-0 ConvTranspose forward (Cin 128, Cout 64; several 64-voxel tiles
    per workgroup, a partial last tile, F.pad ring) is bit-identical to the LDS kernel and
    matches fp64 on the bf16-rounded inputs."""
    L = _lib()
    g = torch.Generator().manual_seed(11)
    N, cin, cout = 2, 128, 64
    x = torch.randn(N, cin, *Sin, generator=g).to(torch.bfloat16)
    w = (torch.randn(cin, cout, 2, 2, 2, generator=g) / math.sqrt(cin)).to(torch.bfloat16)
    b = torch.randn(cout, generator=g)
    u = F.conv_transpose3d(x.double(), w.double(), b.double(), stride=2)
    dz, dyy, dxx = (Sout[i] - u.shape[2 + i] for i in range(3))
    ref = F.pad(u, [dxx // 2, dxx - dxx // 2, dyy // 2, dyy - dyy // 2, dz // 2, dz - dz // 2])
    fp = torch.empty(L.query("pcms_convt_pack_elems", 1, cin, cout), dtype=torch.bfloat16, device=DEV)
    L.call("pcms_convt_pack", 1, w.float().to(DEV), fp, cin, cout, 0)
    xd = ndhwc(x).to(DEV)
    outs = []
    old = L.query("pcms_convt_fwd_stream", -1)
    try:
        for on in (1, 0):
            L.query("pcms_convt_fwd_stream", on)
            o = torch.full((N, *Sout, cout), float("nan"), dtype=torch.bfloat16, device=DEV)
            L.call("pcms_convt_fwd", 1, xd, fp, b.to(DEV), o, N, *Sin, cin, cout, *Sout)
            outs.append(o)
    finally:
        L.query("pcms_convt_fwd_stream", old)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    close(ncdhw(outs[0].cpu()), ref, 1e-2, "convT stream fwd")


@pytest.mark.parametrize("dt,code,tol", DTS)
@pytest.mark.parametrize("ncls", [1, 2])
def test_head(dt, code, tol, ncls):
    L = _lib()
    g = torch.Generator().manual_seed(1)
    N, S = 2, (5, 6, 7)
    a = torch.relu(torch.randn(N, 64, *S, generator=g)).to(dt)
    w = torch.randn(ncls, 64, 1, 1, 1, generator=g) * 0.1
    b = torch.randn(ncls, generator=g)
    ar = a.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    out = F.conv3d(ar, wr, br)
    dl = torch.randn(out.shape, generator=g)
    out.backward(dl.double())
    V = S[0] * S[1] * S[2]
    logits = torch.empty(N, ncls, *S, device=DEV)
    ad = ndhwc(a).to(DEV)
    L.call("pcms_head_fwd", code, ad, w.reshape(ncls, 64).to(DEV), b.to(DEV), logits, V, N, ncls, 0, 0.5)
    probs = torch.empty_like(logits)
    mask = torch.empty_like(logits)
    L.call("pcms_head_fwd", code, ad, w.reshape(ncls, 64).to(DEV), b.to(DEV), probs, V, N, ncls, 1, 0.5)
    L.call("pcms_head_fwd", code, ad, w.reshape(ncls, 64).to(DEV), b.to(DEV), mask, V, N, ncls, 2, 0.5)
    da = torch.empty_like(ad)
    dw = torch.zeros(ncls, 64, device=DEV)
    db = torch.zeros(ncls, device=DEV)
    ws = torch.empty(L.query("pcms_head_bwd_ws_floats", V, N, ncls), device=DEV)
    L.call("pcms_head_bwd", code, ad, dl.to(DEV), w.reshape(ncls, 64).to(DEV), da, dw, db, ws, V, N, ncls)
    # fixed-order reduction: a second backward adds exactly the same amounts
    dw2, db2 = torch.zeros_like(dw), torch.zeros_like(db)
    L.call("pcms_head_bwd", code, ad, dl.to(DEV), w.reshape(ncls, 64).to(DEV), da, dw2, db2, ws, V, N, ncls)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    close(logits.cpu(), out.detach(), 1e-5, "head fwd")
    close(probs.cpu(), torch.sigmoid(out.detach()), 1e-6, "head sigmoid (predict)")
    assert torch.equal(mask.cpu(), (torch.sigmoid(logits.cpu()) > 0.5).float())
    close(ncdhw(da.cpu()), ar.grad, tol, "head dgrad")
    close(dw.cpu(), wr.grad.reshape(ncls, 64), 1e-5, "head wgrad")
    close(db.cpu(), br.grad, 1e-5, "head bias grad")


@pytest.mark.parametrize("dt,code,tol,shift", [d + (0.3,) for d in DTS] + [DTS[0] + (100.0,)])
@pytest.mark.parametrize("ncls", [1, 2])
def test_head_bn_fused(dt, code, tol, shift, ncls):
    """The last decoder block's BN + ReLU fused into the head (pcms_head_bn_fwd / _bwd) vs
    the unfused sequence (pcms_bn_relu -> pcms_head_fwd; pcms_head_bwd -> pcms_bn_relu_bwd):
    bit-identical logits and head weight / bias gradients, the BatchNorm gradients and dy
    equal up to the BN partial sums' order; and both against fp64 autograd of
    relu(batch_norm(y)) -> conv1x1.  ``shift`` 100 (fp32): |mean| / std = 50, where an
    uncentred apply (A y + B) loses ~eps |mean| / std to cancellation."""
    L = _lib()
    g = torch.Generator().manual_seed(4)
    N, S, C = 2, (6, 5, 8), 64
    V = S[0] * S[1] * S[2]
    nvox = N * V
    y = (torch.randn(N, C, *S, generator=g) * 2 + shift).to(dt)
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.1
    w = torch.randn(ncls, 64, 1, 1, 1, generator=g) * 0.1
    b = torch.randn(ncls, generator=g)
    dl = torch.randn(N, ncls, *S, generator=g)
    # fp64 reference
    yr = y.double().requires_grad_(True)
    gr, brr = gamma.double().requires_grad_(True), beta.double().requires_grad_(True)
    wr, br = w.double().requires_grad_(True), b.double().requires_grad_(True)
    out = F.conv3d(F.relu(F.batch_norm(yr, None, None, gr, brr, True, 0.1, 1e-5)), wr, br)
    out.backward(dl.double())
    # device: BN statistics -> scale / shift / mean / invstd (pcms_bn_finalize from exact partials)
    yd = ndhwc(y).to(DEV)
    m = y.double().mean((0, 2, 3, 4))
    var = y.double().var((0, 2, 3, 4), unbiased=False)
    inv = 1.0 / torch.sqrt(var + 1e-5)
    sc = (gamma.double() * inv).float().to(DEV)
    sh = (beta.double() - m * gamma.double() * inv).float().to(DEV)
    mean, invstd = m.float().to(DEV), inv.float().to(DEV)
    W2, bd, dld = w.reshape(ncls, 64).to(DEV), b.to(DEV), dl.to(DEV)
    gd = gamma.to(DEV)
    # unfused
    a = torch.empty_like(yd)
    L.call("pcms_bn_relu", code, yd, a, sc, sh, C, nvox)
    lg0 = torch.empty(N, ncls, *S, device=DEV)
    L.call("pcms_head_fwd", code, a, W2, bd, lg0, V, N, ncls, 0, 0.5)
    ws = torch.empty(L.query("pcms_head_bwd_ws_floats", V, N, ncls), device=DEV)
    da = torch.empty_like(yd)
    dw0, db0 = torch.zeros(ncls, 64, device=DEV), torch.zeros(ncls, device=DEV)
    L.call("pcms_head_bwd", code, a, dld, W2, da, dw0, db0, ws, V, N, ncls)
    rows = max(L.query("pcms_bn_bwd_rows", code, C, nvox), L.query("pcms_head_bn_bwd_rows", V, N))
    part = torch.empty(rows * C * 2, device=DEV)
    coef = torch.empty(3 * C, device=DEV)
    bnws = torch.empty(L.query("pcms_bn_ws_doubles", C), dtype=torch.float64, device=DEV)
    dg0, dbt0 = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
    dy0 = torch.empty_like(yd)
    L.call("pcms_bn_relu_bwd", code, da, yd, sc, sh, mean, invstd, gd, part, coef, dg0, dbt0, dy0, C, nvox, bnws)
    # fused
    lg1 = torch.empty_like(lg0)
    L.call("pcms_head_bn_fwd", code, yd, sc, sh, W2, bd, lg1, V, N, ncls, 0, 0.5)
    dw1, db1 = torch.zeros_like(dw0), torch.zeros_like(db0)
    dg1, dbt1 = torch.zeros_like(dg0), torch.zeros_like(dbt0)
    dy1 = torch.full_like(yd, float("nan"))
    L.call("pcms_head_bn_bwd", code, yd, sc, sh, mean, invstd, gd, dld, W2, dw1, db1, ws, part, coef, dg1, dbt1,
           dy1, V, N, ncls, bnws)
    torch.cuda.synchronize()
    assert torch.equal(lg0, lg1)
    assert torch.equal(dw0, dw1) and torch.equal(db0, db1)
    close(dg1.cpu(), dg0.cpu(), 1e-5, "dgamma fused vs unfused")
    close(dbt1.cpu(), dbt0.cpu(), 1e-5, "dbeta fused vs unfused")
    close(ncdhw(dy1.cpu()), ncdhw(dy0.cpu()), 1e-5 if not code else 1e-2, "dy fused vs unfused")
    close(lg1.cpu(), out.detach(), 1e-5 if not code else 2e-2, "fused logits vs fp64")
    close(ncdhw(dy1.cpu()), yr.grad, 1e-4 if not code else 3e-2, "fused dy vs fp64")
    close(dg1.cpu(), gr.grad, 1e-4 if not code else 3e-2, "fused dgamma vs fp64")
    close(dbt1.cpu(), brr.grad, 1e-4 if not code else 3e-2, "fused dbeta vs fp64")
    close(dw1.cpu(), wr.grad.reshape(ncls, 64), 1e-5 if not code else 2e-2, "fused head wgrad vs fp64")


@pytest.mark.parametrize("wb,wd", [(0.0, 1.0), (0.5, 0.5)])
def test_loss(wb, wd):
    L = _lib()
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, 1, 9, 10, 11, generator=g) * 3
    t = (torch.rand(x.shape, generator=g) < 0.3).float()
    xr = x.double().requires_grad_(True)
    p = torch.sigmoid(xr).reshape(-1)
    tt = t.double().reshape(-1)
    dice = 1 - (2 * (p * tt).sum() + 1) / (p.sum() + tt.sum() + 1)
    ref = wb * F.binary_cross_entropy_with_logits(xr, t.double()) + wd * dice
    ref.backward(torch.tensor(0.7, dtype=torch.float64))
    M = x.numel()
    rows = L.query("pcms_loss_rows", M)
    part = torch.empty(rows * 4, device=DEV)
    sums = torch.empty(4, dtype=torch.float64, device=DEV)
    loss = torch.empty((), device=DEV)
    xd, td = x.to(DEV), t.to(DEV)
    L.call("pcms_loss_fwd", xd, td, M, 1.0, wb, wd, part, sums, loss)
    dx = torch.empty_like(xd)
    L.call("pcms_loss_bwd", xd, td, M, sums, 1.0, wb, wd, torch.tensor(0.7, device=DEV), dx)
    torch.cuda.synchronize()
    assert abs(loss.item() - ref.item()) < 1e-6
    close(dx.cpu(), xr.grad, 1e-5, "loss grad")


def test_adam_matches_torch():
    L = _lib()
    g = torch.Generator().manual_seed(4)
    n = 10007
    p0 = torch.randn(n, generator=g)
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=1e-3, weight_decay=1e-5)
    pd = p0.clone().to(DEV)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    for step in range(1, 4):
        gr = torch.randn(n, generator=g)
        pt.grad = gr.clone()
        opt.step()
        L.call("pcms_adam", pd, gr.to(DEV), m, v, n, 1e-3 / (1 - 0.9 ** step), 0.9, 0.999, 1e-8, 1e-5,
               math.sqrt(1 - 0.999 ** step), 1.0, None)
    torch.cuda.synchronize()
    close(pd.cpu(), pt.detach(), 1e-6, "adam")


@pytest.mark.parametrize("dt,code", [(torch.float32, 0), (torch.bfloat16, 1)])
@pytest.mark.parametrize("S", [(3, 4, 5), (3, 3, 5), (16, 16, 8)])
def test_pack_input(dt, code, S):
    """NCDHW fp32 -> NDHWC 8-channel (4-voxel vector path when V % 4 == 0, else scalar)."""
    L = _lib()
    V = S[0] * S[1] * S[2]
    x = torch.rand(2, 5, *S)
    out = torch.full((2, *S, 8), float("nan"), dtype=dt, device=DEV)
    L.call("pcms_pack_input", code, x.to(DEV), out, 2, 5, V, 8)
    torch.cuda.synchronize()
    exp = torch.zeros(2, *S, 8)
    exp[..., :5] = ndhwc(x)
    close(out.cpu(), exp.to(dt), 0, "pack input")


@pytest.mark.parametrize("N,S", [(2, (16, 16, 16)), (1, (9, 10, 11)), (2, (8, 8, 4)), (1, (6, 20, 33)),
                                 (1, (8, 12, 48)), (3, (4, 4, 16)), (1, (32, 32, 32)), (1, (48, 64, 64)),
                                 (2, (32, 64, 64)), (1, (12, 16, 16)), (4, (8, 64, 128))])
@pytest.mark.parametrize("cin,dense", [(5, 16), (5, 0), (3, 16)])
def test_stem_fwd_wgrad_bf16(N, S, cin, dense):
    """Dedicated stem kernels vs torch conv3d on the bf16-rounded input, on the shapes they
    support (pcms_stem_supported; others refuse and the engine takes the general kernels).
    Forward: the K-dense kernel (PCMS_STEM_DENSE, 9 tap rows x 16: the product for <= 5
    channels; also at 3 channels) and the 14-tap-pair kernel; both against fp64, and against
    each other to the fp32 summation-order noise (same bf16 products)."""
    L = _lib()
    sup = L.query("pcms_stem_supported", N, *S)
    # (4, (8, 64, 128)): 4096 boxes, 16 per persistent workgroup of each kernel
    hot = S[0] % 4 == 0 and S[1] % 4 == 0 and S[2] % 16 == 0
    if hot:
        assert sup == 3, (S, sup)
    if sup == 0:
        with pytest.raises(L.HipError):
            L.call("pcms_stem_fwd", None, None, None, None, None, N, *S, 0)
        return
    g = torch.Generator().manual_seed(sum(S))
    x = torch.rand(N, cin, *S, generator=g).to(torch.bfloat16)
    w = (torch.randn(64, cin, 3, 3, 3, generator=g) * 0.2)
    b = torch.randn(64, generator=g)
    xs = torch.zeros(N, 8, *S, dtype=torch.bfloat16)
    xs[:, :cin] = x
    xd = ndhwc(xs).to(DEV)
    xr = x.double()
    wr = w.to(torch.bfloat16).double().requires_grad_(True)
    ref = F.conv3d(xr, wr, b.double(), padding=1)
    dy = torch.randn(ref.shape, generator=g).to(torch.bfloat16)
    ref.backward(dy.double())
    if sup & 1:
        wp = torch.empty(L.query("pcms_stem_pack_elems"), dtype=torch.bfloat16, device=DEV)
        L.call("pcms_stem_pack", w.to(DEV), wp, cin)
        y = torch.empty(N, *S, 64, dtype=torch.bfloat16, device=DEV)
        rows = L.query("pcms_stem_fwd_rows", N, *S)
        stats = torch.zeros(rows * (64 * 2 + 1), device=DEV)
        L.call("pcms_stem_fwd", xd, wp, b.to(DEV), y, stats, N, *S, dense)
        y_other = torch.empty_like(y)
        L.call("pcms_stem_fwd", xd, wp, b.to(DEV), y_other, None, N, *S, 16 - dense)
        torch.cuda.synchronize()
        close(ncdhw(y.cpu()), ref.detach(), 1e-2, "stem fwd")
        # the two K orders round differently only where an fp32 sum lands on a bf16 tie
        assert (y.float() - y_other.float()).abs().max().item() <= 2 ** -6 * ref.abs().max().item()
        mean, var = bn_moments(stats, rows, 64, N * S[0] * S[1] * S[2])
        yr = ref.detach().transpose(0, 1).reshape(64, -1)
        close(mean, yr.mean(1), 1e-3, "stem stats mean")
        close(var, yr.var(1, unbiased=False), 1e-3, "stem stats var")
    if sup & 2:
        guard = 4096
        dw = torch.zeros(64 * cin * 27 + guard, device=DEV)
        ws = torch.empty(L.query("pcms_stem_wgrad_ws_floats", N, *S, cin), device=DEV)
        old = L.query("pcms_stem_wgrad_dense", 1 if dense else 0)  # the weight gradient's column form too
        try:
            L.call("pcms_stem_wgrad", xd, ndhwc(dy).to(DEV), dw, ws, cin, N, *S)
            torch.cuda.synchronize()
        finally:
            L.query("pcms_stem_wgrad_dense", old)
        assert dw[64 * cin * 27:].abs().max().item() == 0.0
        close(dw[:64 * cin * 27].cpu().view(64, cin, 3, 3, 3), wr.grad, 1e-4, "stem wgrad")


@pytest.mark.parametrize("N,S", [(2, (16, 16, 16)), (3, (4, 4, 16)), (1, (12, 16, 32)), (2, (32, 64, 64))])
@pytest.mark.parametrize("dense", [1, 0])
def test_stem_wgrad_bn_fused(N, S, dense):
    """The stem's BatchNorm + ReLU backward apply fused into its weight gradient
    (pcms_stem_wgrad_bn) vs the unfused pair (pcms_bn_relu_bwd's apply pass -> dy in HBM ->
    pcms_stem_wgrad) on the same bf16 inputs -- the in-LDS dy uses the apply kernel's
    arithmetic, so the weight gradients agree to fp32 summation noise -- and vs fp64 autograd of
    conv3d -> batch_norm -> relu."""
    L = _lib()
    assert L.query("pcms_stem_supported", N, *S) & 2
    old = L.query("pcms_stem_wgrad_dense", dense)
    try:
        _stem_wgrad_bn_case(L, N, S)
    finally:
        L.query("pcms_stem_wgrad_dense", old)


def _stem_wgrad_bn_case(L, N, S):
    g = torch.Generator().manual_seed(11 + sum(S))
    nvox = N * S[0] * S[1] * S[2]
    x = torch.rand(N, 5, *S, generator=g).to(torch.bfloat16)
    w = torch.randn(64, 5, 3, 3, 3, generator=g) * 0.2
    gamma = torch.rand(64, generator=g) + 0.5
    beta = torch.randn(64, generator=g) * 0.1
    xs = torch.zeros(N, 8, *S, dtype=torch.bfloat16)
    xs[:, :5] = x
    xd = ndhwc(xs).to(DEV)
    y = F.conv3d(x.double(), w.to(torch.bfloat16).double(), None, padding=1).to(torch.bfloat16)  # stem output
    da = torch.randn(N, 64, *S, generator=g).to(torch.bfloat16)                                  # grad of ReLU out
    # fp64 reference: dW of conv -> BN(train) -> ReLU given y (rounded) and da
    yr = y.double().requires_grad_(True)
    F.relu(F.batch_norm(yr, None, None, gamma.double(), beta.double(), True, 0.1, 1e-5)).backward(da.double())
    # dy is a bf16 tensor in the product as in the unfused path: its rounding is part of the
    # result (dW = sum dy x cancels most of the elements' magnitude: at 2 x 32x64x64 the bf16
    # rounding of dy alone moves dW by several % of its max), so the reference rounds it too
    dw_ref = torch.nn.grad.conv3d_weight(x.double(), (64, 5, 3, 3, 3), yr.grad.to(torch.bfloat16).double(),
                                         padding=1)
    m = y.double().mean((0, 2, 3, 4))
    inv = 1.0 / torch.sqrt(y.double().var((0, 2, 3, 4), unbiased=False) + 1e-5)
    sc = (gamma.double() * inv).float().to(DEV)
    sh = (beta.double() - m * gamma.double() * inv).float().to(DEV)
    mean, invstd, gd = m.float().to(DEV), inv.float().to(DEV), gamma.to(DEV)
    yd, dad = ndhwc(y).to(DEV), ndhwc(da).to(DEV)
    rows = L.query("pcms_bn_bwd_rows", 1, 64, nvox)
    part = torch.empty(rows * 64 * 2, device=DEV)
    coef = torch.empty(3 * 64, device=DEV)
    bnws = torch.empty(L.query("pcms_bn_ws_doubles", 64), dtype=torch.float64, device=DEV)
    ws = torch.empty(L.query("pcms_stem_wgrad_ws_floats", N, *S, 5), device=DEV)
    # unfused
    dg0, db0, dy0 = torch.zeros(64, device=DEV), torch.zeros(64, device=DEV), torch.empty_like(yd)
    L.call("pcms_bn_relu_bwd", 1, dad, yd, sc, sh, mean, invstd, gd, part, coef, dg0, db0, dy0, 64, nvox, bnws)
    dw0 = torch.zeros(64 * 5 * 27, device=DEV)
    L.call("pcms_stem_wgrad", xd, dy0, dw0, ws, 5, N, *S)
    # fused: reduce + finalize only (dy NULL), then the wgrad applies in LDS
    dg1, db1 = torch.zeros(64, device=DEV), torch.zeros(64, device=DEV)
    coef1 = torch.full((3 * 64,), float("nan"), device=DEV)
    L.call("pcms_bn_relu_bwd", 1, dad, yd, sc, sh, mean, invstd, gd, part, coef1, dg1, db1, None, 64, nvox, bnws)
    dw1 = torch.zeros(64 * 5 * 27, device=DEV)
    L.call("pcms_stem_wgrad_bn", xd, dad, yd, sc, sh, mean, invstd, coef1, dw1, ws, 5, N, *S)
    torch.cuda.synchronize()
    assert torch.equal(dg0, dg1) and torch.equal(db0, db1) and torch.equal(coef, coef1)
    # (the in-LDS dy and the apply kernel may contract k1 g + k2 xhat + k3 differently: a rare
    # one-ulp bf16 difference in dy)
    close(dw1.cpu(), dw0.cpu(), 1e-4, "fused vs unfused stem wgrad")
    close(dw1.cpu().view(64, 5, 3, 3, 3), dw_ref, 2e-2, "fused stem wgrad vs fp64")


@pytest.mark.parametrize("cout,cin", [(64, 64), (128, 256), (64, 128), (512, 1024)])
def test_conv3_pack2_equals_two_packs(cout, cin):
    """pcms_conv3_pack2 (forward + dgrad bf16 packs from one weight read) is bit-identical to
    pcms_conv3_pack with flip 0 and flip 1."""
    L = _lib()
    code = 1  # bf16
    ck = L.query("pcms_conv3_chunk", code)
    w = torch.randn(cout, cin, 3, 3, 3, device=DEV)
    f1 = torch.empty(-(-cin // ck) * 27 * cout * ck, dtype=torch.bfloat16, device=DEV)
    d1 = torch.empty(-(-cout // ck) * 27 * cin * ck, dtype=torch.bfloat16, device=DEV)
    f2, d2 = torch.full_like(f1, 7), torch.full_like(d1, 7)
    L.call("pcms_conv3_pack", code, w, f1, cout, cin, 0)
    L.call("pcms_conv3_pack", code, w, d1, cout, cin, 1)
    L.call("pcms_conv3_pack2", code, w, f2, d2, cout, cin)
    torch.cuda.synchronize()
    assert torch.equal(f1.view(torch.int16), f2.view(torch.int16))
    assert torch.equal(d1.view(torch.int16), d2.view(torch.int16))


@pytest.mark.parametrize("flip", [0, 1])
@pytest.mark.parametrize("cout,cin", [(64, 24), (128, 64)])
def test_conv3_pack_x6_layout(flip, cout, cin):
    """fp32 build (bf16x6) weight pack, bit-exact against a torch emulation of the split:
    rows [chunk][27][J][48 bf16] = [h | h] [m | h] [l | m] over 8 k, h = rne(v), m = rne(v - h),
    l = rne(v - h - m); dgrad packs (flip) mirror the taps and swap Cin / Cout."""
    L = _lib()
    code = 0
    w = torch.randn(cout, cin, 27, device=DEV) * 0.1
    J, K = (cin, cout) if flip else (cout, cin)
    n = L.query("pcms_conv3_pack_elems", code, J, K)
    out = torch.full((n,), float("nan"), device=DEV)
    L.call("pcms_conv3_pack", code, w, out, cout, cin, flip)
    torch.cuda.synchronize()
    nch = -(-K // 8)
    got = out.view(torch.int16)[: nch * 27 * J * 48].view(nch, 27, J, 48).cpu()
    wc = w.cpu()
    src = wc.permute(1, 0, 2).flip(2) if flip else wc  # [J][K][27]
    src = torch.nn.functional.pad(src, (0, 0, 0, nch * 8 - K))  # zero k padding
    v = src.view(J, nch, 8, 27).permute(1, 3, 0, 2)  # [chunk][t][J][k]
    h = v.to(torch.bfloat16)
    r = v - h.float()
    m = r.to(torch.bfloat16)
    lo = (r - m.float()).to(torch.bfloat16)
    exp = torch.cat([h, h, m, h, lo, m], dim=3).view(torch.int16)
    assert torch.equal(got, exp)


@pytest.mark.parametrize("N,S,C,wgs", [(2, (32, 32, 32), 64, 0), (1, (32, 32, 32), 128, 24)])
def test_bnin_conv_and_wgrad_bit_identical(N, S, C, wgs):
    """The BatchNorm + ReLU of a DoubleConv's first conv applied inside its second conv's
    staging (pcms_conv3_fwd_bnin / pcms_conv3_wgrad_bnin: models/unet3d.py:31-35) against the
    stored a1 = pcms_bn_relu(y1) fed to pcms_conv3_fwd / pcms_conv3_wgrad: bit-identical outputs,
    BatchNorm partials and weight gradients (the same bn_relu1 arithmetic and bf16 rounding);
    padding stays zero (relu(0 * sc + sh) would not be).  wgs > 0: a persistent grid smaller
    than the box count (several boxes per workgroup)."""
    L = _lib()
    old = L.query("pcms_conv3_big_min_boxes", 1)
    old_w = L.query("pcms_conv3_big_max_wgs", wgs)
    try:
        assert L.query("pcms_conv3_bnin_ok", N, *S, C, C, 256) == 1
        g = torch.Generator().manual_seed(21)
        nvox = N * S[0] * S[1] * S[2]
        T = torch.bfloat16
        y1 = (torch.randn(nvox * C, generator=g) * 2).to(T).to(DEV)
        sc = (torch.rand(C, generator=g) + 0.5).to(DEV)
        sh = (torch.randn(C, generator=g) * 0.5).to(DEV)  # positive shifts: padding must not become relu(sh)
        w = (torch.randn(C, C, 27, generator=g) * 0.05).to(DEV)
        wp = torch.empty(L.query("pcms_conv3_pack_elems", 1, C, C), dtype=T, device=DEV)
        L.call("pcms_conv3_pack", 1, w, wp, C, C, 0)
        bias = torch.randn(C, generator=g).to(DEV)
        dy = (torch.randn(nvox * C, generator=g)).to(T).to(DEV)
        rows = L.query("pcms_conv3_fwd_rows", 1, N, *S, C, 0, C)
        a1 = torch.empty_like(y1)
        L.call("pcms_bn_relu", 1, y1, a1, sc, sh, C, nvox)
        out = []
        for fused in (False, True):
            y = torch.full_like(y1, float("nan"))
            st = torch.full((rows * (2 * C + 1),), float("nan"), device=DEV)
            dw = torch.zeros(C * C * 27, device=DEV)
            dwt = torch.empty(max(1, L.query("pcms_conv3_wgrad_ws_floats", 1, N, *S, C, 0, C, 256)), device=DEV)
            if fused:
                L.call("pcms_conv3_fwd_bnin", 1, y1, C, sc, sh, wp, bias, y, st, N, *S, C)
                L.call("pcms_conv3_wgrad_bnin", 1, y1, C, sc, sh, dy, dw, dwt, N, *S, C, C, 256, 0)
            else:
                L.call("pcms_conv3_fwd", 1, a1, C, None, 0, wp, bias, y, None, C, None, st, 0, N, *S, C, 1)
                L.call("pcms_conv3_wgrad", 1, a1, C, None, 0, dy, dw, dwt, N, *S, C, C, 256, 0)
            torch.cuda.synchronize()
            out.append((y.view(torch.int16).clone(), st.clone(), dw.clone()))
        (y0, s0, d0), (y1_, s1, d1) = out
        assert torch.equal(y0, y1_)
        assert torch.equal(s0, s1)
        assert torch.equal(d0, d1)
        # and against fp64 on the rounded activation (the fused forward computes the same conv)
        a64 = ncdhw(a1.view(N, *S, C).cpu()).double()
        ref = F.conv3d(a64, w.view(C, C, 3, 3, 3).cpu().double(), bias.cpu().double(), padding=1)
        close(ncdhw(y1_.view(T).view(N, *S, C).cpu()), ref, 1e-2, "fused conv vs fp64")
    finally:
        L.query("pcms_conv3_big_min_boxes", old)
        L.query("pcms_conv3_big_max_wgs", old_w)


def _pack16(L, w, cout, cin, fwd=True, dgrad=True):
    """pcms_conv3_pack16 of one conv (a one-row table): (fwd16, dgrad16) device tensors."""
    T = torch.bfloat16
    f = torch.empty(L.query("pcms_conv3_pack16_elems", cout, cin), dtype=T, device=DEV) if fwd else None
    d = torch.empty(L.query("pcms_conv3_pack16_elems", cin, cout), dtype=T, device=DEV) if dgrad else None
    wd = w.reshape(-1).to(DEV).contiguous()
    tab = torch.tensor([[wd.data_ptr(), cout, cin, f.data_ptr() if f is not None else 0,
                         d.data_ptr() if d is not None else 0, 0, 0, 0]], dtype=torch.int64, device=DEV)
    L.call("pcms_conv3_pack16", tab, 1, (cout // 32) * (cin // 32))
    torch.cuda.synchronize()
    return f, d


@pytest.mark.parametrize("nt8", [1, 0])
@pytest.mark.parametrize("N,c0,c1,cout,cy0,S,wgs", [
    (1, 64, 0, 64, 64, (8, 8, 16), 0),         # one box
    (2, 32, 32, 128, 64, (16, 8, 32), 0),      # dual source, two-pointer output, 2 channel blocks
    (1, 16, 48, 64, 64, (8, 16, 16), 0),       # chunks split unevenly between the sources
    (1, 128, 0, 192, 128, (16, 16, 16), 0),    # odd number of 64-channel blocks, split output
    (2, 64, 0, 64, 64, (16, 16, 32), 3),       # persistent: 3 slots walk 16 boxes (6, 5, 5)
    (2, 32, 32, 128, 64, (16, 16, 32), 4),     # 2 slots x 2 channel blocks, 8 boxes each
    (1, 64, 64, 64, 64, (16, 24, 16), 5),      # dual source, 5 slots over 6 boxes (2 + 1 x 4)
    (1, 64, 0, 256, 128, (8, 16, 16), 3),      # 128-channel blocks (nt8): 2 blocks, split output
])
def test_conv3_fwd16_big_box(nt8, N, c0, c1, cout, cy0, S, wgs):
    """The 16x16x32 big-box kernel (pcms_conv3_fwd16, tap pairs x 16 channels per MFMA, the
    pack16 weights) on the big-box cases: vs torch conv3d in fp64 on the same bf16 inputs, the
    BN partial moments, and within bf16 rounding of the 32x32x16 big-box kernel's output.
    nt8 1: 128-channel outputs run as 128-channel blocks on 4-deep boxes (B6G<4, 8>)."""
    L = _lib()
    old = L.query("pcms_conv3_big_min_boxes", 1)
    old_w = L.query("pcms_conv3_big_max_wgs", wgs)
    old_nt = L.query("pcms_conv3_b16_nt8", nt8)
    try:
        dt = torch.bfloat16
        g = torch.Generator().manual_seed(c0 + 5 * c1 + cout)
        x0 = torch.randn(N, c0, *S, generator=g).to(dt)
        x1 = torch.randn(N, c1, *S, generator=g).to(dt)
        cin = c0 + c1
        w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)
        b = torch.randn(cout, generator=g)
        ref = F.conv3d(torch.cat([x0, x1], 1).double(), w.to(dt).double(), b.double(), padding=1)
        assert L.query("pcms_conv3_big16_ok", N, *S, c0, c1, cout) == 1
        w16, _ = _pack16(L, w, cout, cin, dgrad=False)
        wp = torch.empty(L.query("pcms_conv3_pack_elems", 1, cout, cin), dtype=dt, device=DEV)
        L.call("pcms_conv3_pack", 1, w.to(DEV), wp, cout, cin, 0)
        nvox = N * S[0] * S[1] * S[2]
        outs = []
        for k16 in (True, False):
            rows = L.query("pcms_conv3_fwd16_rows" if k16 else "pcms_conv3_fwd_rows", *([] if k16 else [1]), N, *S,
                           c0, c1, cout)
            y0 = torch.full((N, *S, cy0), float("nan"), dtype=dt, device=DEV)
            y1 = torch.full((N, *S, max(cout - cy0, 8)), float("nan"), dtype=dt, device=DEV)
            stats = torch.full((rows * (cout * 2 + 1),), float("nan"), device=DEV)
            xa, xb = ndhwc(x0).to(DEV), ndhwc(x1).to(DEV) if c1 else None
            if k16:
                L.call("pcms_conv3_fwd16", xa, c0, xb, c1, None, None, w16, b.to(DEV), y0,
                       y1 if cout > cy0 else None, cy0, stats, 0, N, *S, cout)
            else:
                L.call("pcms_conv3_fwd", 1, xa, c0, xb, c1, wp, b.to(DEV), y0, y1 if cout > cy0 else None, cy0, None,
                       stats, 0, N, *S, cout, 1)
            torch.cuda.synchronize()
            got = ncdhw(y0.cpu())
            if cout > cy0:
                got = torch.cat([got, ncdhw(y1.cpu())], 1)
            outs.append(got)
            close(got, ref, 1e-2, f"big-box fwd ({'16x16x32' if k16 else '32x32x16'})")
            mean, var = bn_moments(stats, rows, cout, nvox)
            yref = ref.transpose(0, 1).reshape(cout, -1)
            close(mean, yref.mean(1), 1e-3, "stats mean")
            close(var, yref.var(1, unbiased=False), 1e-3, "stats var")
        close(outs[0], outs[1].double(), 1e-2, "16x16x32 vs 32x32x16")
    finally:
        L.query("pcms_conv3_big_min_boxes", old)
        L.query("pcms_conv3_big_max_wgs", old_w)
        L.query("pcms_conv3_b16_nt8", old_nt)


@pytest.mark.parametrize("N,c0,c1,cout,cy0,S,wgs", [
    (1, 64, 0, 64, 64, (12, 8, 16), 0),        # 3 four-deep boxes
    (2, 32, 32, 128, 64, (4, 16, 32), 0),      # dual source, two-pointer output, 2 channel blocks
    (1, 128, 0, 192, 128, (12, 16, 16), 4),    # 3 channel blocks x 1 slot walking 6 boxes
    (2, 16, 16, 64, 64, (20, 8, 16), 3),       # 3 slots over 10 boxes
])
def test_conv3_fwd16_four_deep(N, c0, c1, cout, cy0, S, wgs):
    """pcms_conv3_fwd16 on boxes of 4 d-planes (4 waves, one workgroup per CU: the level-2
    shapes, where 8-deep boxes leave CUs idle; D % 8 != 0 here so the 4-deep form is the one
    that runs): vs torch conv3d in fp64 on the same bf16 inputs, and its BN partial moments
    (pcms_conv3_fwd16_rows rows)."""
    L = _lib()
    old = L.query("pcms_conv3_big_min_boxes", 1)
    old_w = L.query("pcms_conv3_big_max_wgs", wgs)
    try:
        dt = torch.bfloat16
        g = torch.Generator().manual_seed(3 * c0 + 7 * c1 + cout)
        x0 = torch.randn(N, c0, *S, generator=g).to(dt)
        x1 = torch.randn(N, c1, *S, generator=g).to(dt)
        cin = c0 + c1
        w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)
        b = torch.randn(cout, generator=g)
        ref = F.conv3d(torch.cat([x0, x1], 1).double(), w.to(dt).double(), b.double(), padding=1)
        assert L.query("pcms_conv3_big16_ok", N, *S, c0, c1, cout) == 1
        w16, _ = _pack16(L, w, cout, cin, dgrad=False)
        nvox = N * S[0] * S[1] * S[2]
        rows = L.query("pcms_conv3_fwd16_rows", N, *S, c0, c1, cout)
        nbox = N * (S[0] // 4) * (S[1] // 8) * (S[2] // 16)
        assert 1 <= rows <= nbox
        y0 = torch.full((N, *S, cy0), float("nan"), dtype=dt, device=DEV)
        y1 = torch.full((N, *S, max(cout - cy0, 8)), float("nan"), dtype=dt, device=DEV)
        stats = torch.full((rows * (cout * 2 + 1),), float("nan"), device=DEV)
        xa, xb = ndhwc(x0).to(DEV), ndhwc(x1).to(DEV) if c1 else None
        L.call("pcms_conv3_fwd16", xa, c0, xb, c1, None, None, w16, b.to(DEV), y0, y1 if cout > cy0 else None, cy0,
               stats, 0, N, *S, cout)
        torch.cuda.synchronize()
        got = ncdhw(y0.cpu())
        if cout > cy0:
            got = torch.cat([got, ncdhw(y1.cpu())], 1)
        close(got, ref, 1e-2, "four-deep fwd16")
        mean, var = bn_moments(stats, rows, cout, nvox)
        yref = ref.transpose(0, 1).reshape(cout, -1)
        close(mean, yref.mean(1), 1e-3, "stats mean")
        close(var, yref.var(1, unbiased=False), 1e-3, "stats var")
        # the dgrad direction on the same boxes (pack16 dgrad form) and the fused input BN + ReLU
        if c1 == 0:
            _, d16 = _pack16(L, w, cout, cin, fwd=False)
            dy = torch.randn(N, cout, *S, generator=g).to(dt)
            dx = torch.empty(N, *S, cin, dtype=dt, device=DEV)
            L.call("pcms_conv3_fwd16", ndhwc(dy).to(DEV), cout, None, 0, None, None, d16, None, dx, None, cin, None,
                   0, N, *S, cin)
            torch.cuda.synchronize()
            close(ncdhw(dx.cpu()), F.conv_transpose3d(dy.double(), w.to(dt).double(), padding=1), 1e-2,
                  "four-deep dgrad16")
            sc = (torch.rand(cin, generator=g) + 0.5).to(DEV)
            sh = (torch.randn(cin, generator=g) * 0.5).to(DEV)
            a = torch.empty_like(xa)
            L.call("pcms_bn_relu", 1, xa, a, sc, sh, cin, nvox)
            outs = []
            for fused in (False, True):
                y = torch.full((N, *S, cout), float("nan"), dtype=dt, device=DEV)
                st = torch.full((rows * (cout * 2 + 1),), float("nan"), device=DEV)
                L.call("pcms_conv3_fwd16", xa if fused else a, c0, None, 0, sc if fused else None,
                       sh if fused else None, w16, b.to(DEV), y, None, cout, st, 0, N, *S, cout)
                torch.cuda.synchronize()
                outs.append((y.view(torch.int16).clone(), st.clone()))
            assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    finally:
        L.query("pcms_conv3_big_min_boxes", old)
        L.query("pcms_conv3_big_max_wgs", old_w)


@pytest.mark.parametrize("N,c0,c1,cout,S", [
    (2, 64, 0, 128, (8, 16, 8)),       # 4 boxes x 2 channel blocks, 4 splits of 1 chunk
    (2, 128, 128, 128, (4, 16, 8)),    # dual source (the chunks of a split may span both)
    (1, 256, 0, 64, (16, 32, 16)),     # 16 boxes x 1 channel block, 16 chunks in 16 splits
])
def test_conv3_fwd16_split(N, c0, c1, cout, S):
    """The level-3 split-K form of the 16x16x32 kernel (4 d x 16 h x 8 w boxes, fp32 partial
    rows per split) summed by pcms_split_epilogue: bf16 output and BN moments vs torch conv3d
    in fp64 on the same bf16 inputs; and the dgrad direction (dgrad pack16, split output)."""
    L = _lib()
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(5 * c0 + c1 + cout)
    cin = c0 + c1
    x0 = torch.randn(N, c0, *S, generator=g).to(dt)
    x1 = torch.randn(N, c1, *S, generator=g).to(dt)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cin)
    b = torch.randn(cout, generator=g)
    sp = L.query("pcms_conv3_fwd16_split_ok", N, *S, c0, c1, cout)
    assert sp >= 2
    w16, d16 = _pack16(L, w, cout, cin)
    nvox = N * S[0] * S[1] * S[2]
    acc = torch.full((sp * nvox * cout,), float("nan"), device=DEV)
    L.call("pcms_conv3_fwd16_split", ndhwc(x0).to(DEV), c0, ndhwc(x1).to(DEV) if c1 else None, c1, w16, acc,
           N, *S, cout, sp)
    y = torch.empty(N, *S, cout, dtype=dt, device=DEV)
    rows = L.query("pcms_split_epilogue_rows", nvox)
    stats = torch.full((rows * (cout * 2 + 1),), float("nan"), device=DEV)
    L.call("pcms_split_epilogue", 1, acc, sp, b.to(DEV), y, None, cout, stats, cout, nvox, 0)
    torch.cuda.synchronize()
    ref = F.conv3d(torch.cat([x0, x1], 1).double(), w.to(dt).double(), b.double(), padding=1)
    close(ncdhw(y.cpu()), ref, 1e-2, "fwd16 split")
    mean, var = bn_moments(stats, rows, cout, nvox)
    yref = ref.transpose(0, 1).reshape(cout, -1)
    close(mean, yref.mean(1), 1e-3, "stats mean")
    close(var, yref.var(1, unbiased=False), 1e-3, "stats var")
    # dgrad: dx = conv(dy, w transposed, flipped), split into two outputs at cin / 2
    spd = L.query("pcms_conv3_fwd16_split_ok", N, *S, cout, 0, cin)
    if spd:
        dy = torch.randn(N, cout, *S, generator=g).to(dt)
        accd = torch.full((spd * nvox * cin,), float("nan"), device=DEV)
        L.call("pcms_conv3_fwd16_split", ndhwc(dy).to(DEV), cout, None, 0, d16, accd, N, *S, cin, spd)
        cy0 = cin // 2 if cin >= 128 else cin
        o0 = torch.empty(N, *S, cy0, dtype=dt, device=DEV)
        o1 = torch.empty(N, *S, max(cin - cy0, 8), dtype=dt, device=DEV)
        L.call("pcms_split_epilogue", 1, accd, spd, None, o0, o1 if cin > cy0 else None, cy0, None, cin, nvox, 0)
        torch.cuda.synchronize()
        got = ncdhw(o0.cpu())
        if cin > cy0:
            got = torch.cat([got, ncdhw(o1.cpu())], 1)
        close(got, F.conv_transpose3d(dy.double(), w.to(dt).double(), padding=1), 1e-2, "dgrad16 split")


@pytest.mark.parametrize("nt8", [1, 0])
@pytest.mark.parametrize("N,cout,cin,S,wgs", [(2, 64, 64, (16, 16, 32), 0), (1, 64, 128, (16, 16, 16), 3),
                                              (2, 128, 64, (8, 16, 32), 0), (1, 64, 256, (8, 8, 16), 0)])
def test_conv3_dgrad16(nt8, N, cout, cin, S, wgs):
    """The dgrad direction on the 16x16x32 kernel (pack16 dgrad form: rows Cin, k Cout, taps
    mirrored): dx = conv(dy, w transposed and flipped) vs fp64, and the split output of a
    dgrad into the two Up3D sources (cy0)."""
    L = _lib()
    old = L.query("pcms_conv3_big_min_boxes", 1)
    old_w = L.query("pcms_conv3_big_max_wgs", wgs)
    old_nt = L.query("pcms_conv3_b16_nt8", nt8)
    try:
        dt = torch.bfloat16
        g = torch.Generator().manual_seed(cout * 7 + cin)
        dy = torch.randn(N, cout, *S, generator=g).to(dt)
        w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(27 * cout)
        ref = F.conv_transpose3d(dy.double(), w.to(dt).double(), padding=1)
        _, d16 = _pack16(L, w, cout, cin, fwd=False)
        cy0 = cin // 2 if cin >= 128 else cin
        y0 = torch.empty(N, *S, cy0, dtype=dt, device=DEV)
        y1 = torch.empty(N, *S, max(cin - cy0, 8), dtype=dt, device=DEV)
        L.call("pcms_conv3_fwd16", ndhwc(dy).to(DEV), cout, None, 0, None, None, d16, None, y0,
               y1 if cin > cy0 else None, cy0, None, 0, N, *S, cin)
        torch.cuda.synchronize()
        got = ncdhw(y0.cpu())
        if cin > cy0:
            got = torch.cat([got, ncdhw(y1.cpu())], 1)
        close(got, ref, 1e-2, "dgrad16")
    finally:
        L.query("pcms_conv3_big_min_boxes", old)
        L.query("pcms_conv3_big_max_wgs", old_w)
        L.query("pcms_conv3_b16_nt8", old_nt)


@pytest.mark.parametrize("N,S,C,wgs", [(2, (32, 32, 32), 64, 0), (1, (32, 32, 32), 128, 24), (1, (16, 16, 32), 128, 0)])
def test_bnin_conv16_bit_identical(N, S, C, wgs):
    """pcms_conv3_fwd16 with the input BatchNorm + ReLU in its staging (isc / ish) against the
    same kernel on the stored a1 = pcms_bn_relu(y1): bit-identical outputs and BN partials;
    padding stays zero."""
    L = _lib()
    old = L.query("pcms_conv3_big_min_boxes", 1)
    old_w = L.query("pcms_conv3_big_max_wgs", wgs)
    try:
        g = torch.Generator().manual_seed(22)
        nvox = N * S[0] * S[1] * S[2]
        T = torch.bfloat16
        y1 = (torch.randn(nvox * C, generator=g) * 2).to(T).to(DEV)
        sc = (torch.rand(C, generator=g) + 0.5).to(DEV)
        sh = (torch.randn(C, generator=g) * 0.5).to(DEV)
        w = (torch.randn(C, C, 27, generator=g) * 0.05)
        w16, _ = _pack16(L, w, C, C, dgrad=False)
        bias = torch.randn(C, generator=g).to(DEV)
        rows = L.query("pcms_conv3_fwd16_rows", N, *S, C, 0, C)
        a1 = torch.empty_like(y1)
        L.call("pcms_bn_relu", 1, y1, a1, sc, sh, C, nvox)
        out = []
        for fused in (False, True):
            y = torch.full_like(y1, float("nan"))
            st = torch.full((rows * (2 * C + 1),), float("nan"), device=DEV)
            if fused:
                L.call("pcms_conv3_fwd16", y1, C, None, 0, sc, sh, w16, bias, y, None, C, st, 0, N, *S, C)
            else:
                L.call("pcms_conv3_fwd16", a1, C, None, 0, None, None, w16, bias, y, None, C, st, 0, N, *S, C)
            torch.cuda.synchronize()
            out.append((y.view(torch.int16).clone(), st.clone()))
        assert torch.equal(out[0][0], out[1][0])
        assert torch.equal(out[0][1], out[1][1])
        a64 = ncdhw(a1.view(N, *S, C).cpu()).double()
        ref = F.conv3d(a64, w.view(C, C, 3, 3, 3).to(T).double(), bias.cpu().double(), padding=1)
        close(ncdhw(out[1][0].view(T).view(N, *S, C).cpu()), ref, 1e-2, "fused conv16 vs fp64")
    finally:
        L.query("pcms_conv3_big_min_boxes", old)
        L.query("pcms_conv3_big_max_wgs", old_w)
