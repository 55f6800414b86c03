"""The step variants of the reference's other trainers:

* grad clip: ``torch.nn.utils.clip_grad_norm_(params, max_norm=1.0)`` before Adam
  (train_bph.py:166, train_bph_cv.py:311) -> pcms_grad_clip (fused norm, coefficient folded
  into the Adam kernel, or applied in place by ``pcms_amd.amp.clip_grad_norm_``);
* mixed precision: ``GradScaler('cuda')`` + ``scaler.scale(loss).backward();
  scaler.step(opt); scaler.update()`` (train_bph_optimized.py:248-298);
* K-fold splits: ``get_kfold_splits`` = sklearn KFold(shuffle, random_state=42)
  (script/data_loader.py:468-497).
"""
import math
import os

import numpy as np
import pytest
import torch


def test_kfold_matches_sklearn():
    from sklearn.model_selection import KFold
    from pcms_amd.data import kfold_indices
    for n, k in [(10, 5), (23, 5), (7, 3), (5, 5)]:
        ours = kfold_indices(n, k)
        ref = list(KFold(n_splits=k, shuffle=True, random_state=42).split(range(n)))
        assert len(ours) == len(ref)
        for (a_tr, a_va), (b_tr, b_va) in zip(ours, ref):
            assert np.array_equal(a_tr, b_tr) and np.array_equal(a_va, b_va)
    with pytest.raises(ValueError):
        kfold_indices(3, 5)


def test_get_kfold_splits_scans_case_list(tmp_path):
    from pcms_amd.data import get_kfold_splits, write_nifti
    adc = tmp_path / "BPH-PCA" / "BPH" / "ADC"
    adc.mkdir(parents=True)
    for i in range(6):
        write_nifti(str(adc / f"case{i}.nii"), np.zeros((2, 2, 2), np.float32))
    splits = get_kfold_splits(str(tmp_path), n_splits=3)
    assert len(splits) == 3
    assert sorted(np.concatenate([va for _, va in splits]).tolist()) == list(range(6))


def _model_and_grads(seed=0):
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    torch.manual_seed(seed)
    m = UNet3D(n_modalities=5, n_classes=1, precision="fp32").cuda()
    opt = FlatAdam(m, lr=1e-4, weight_decay=1e-5)
    gen = torch.Generator().manual_seed(5)
    x = torch.rand(2, 5, 16, 16, 16, generator=gen).cuda()
    y = (torch.rand(2, 1, 16, 16, 16, generator=gen) < 0.5).float().cuda()
    opt.zero_grad()
    BCEDiceLoss()(m(x), y).backward()
    return m, opt


@pytest.mark.gpu
@pytest.mark.parametrize("max_norm", [1e-3, 1e6])
def test_clip_grad_norm_matches_torch(max_norm):
    """clip_grad_norm_ semantics: total 2-norm over every gradient, coefficient
    min(1, max_norm / (norm + 1e-6)) applied in place.  The reference norm is taken in fp64
    (torch's own fp32 per-tensor CPU norms carry ~1e-4 relative summation error over these
    multi-million-element tensors; the kernel sums fp64 partials)."""
    from pcms_amd.amp import clip_grad_norm_
    m, _ = _model_and_grads()
    g = [p.grad.detach().cpu().clone() for p in m.parameters()]
    ref_norm = float(torch.cat([t.double().reshape(-1) for t in g]).norm())
    coef = min(1.0, max_norm / (ref_norm + 1e-6))
    # torch's own function on the same gradients agrees within its fp32 summation error
    ref_params = [torch.zeros_like(t, requires_grad=True) for t in g]
    for p, t in zip(ref_params, g):
        p.grad = t.clone()
    assert abs(float(torch.nn.utils.clip_grad_norm_(ref_params, max_norm=max_norm)) - ref_norm) <= 1e-3 * ref_norm
    norm = clip_grad_norm_(m, max_norm)
    torch.cuda.synchronize()
    assert abs(float(norm) - ref_norm) <= 1e-6 * ref_norm
    for p, t in zip(m.parameters(), g):
        torch.testing.assert_close(p.grad.cpu(), t * coef, rtol=2e-6, atol=1e-12)


@pytest.mark.gpu
def test_trainer_clip_step_equals_clip_then_adam():
    """Trainer(max_grad_norm=1.0).step == backward, clip_grad_norm_(1.0), Adam (the clip
    coefficient folded into the Adam kernel instead of an extra pass)."""
    from pcms_amd.amp import clip_grad_norm_
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    from pcms_amd.utils.trainer import Trainer
    gen = torch.Generator().manual_seed(9)
    batch = {"image": torch.rand(2, 5, 16, 16, 16, generator=gen),
             "label": (torch.rand(2, 1, 16, 16, 16, generator=gen) < 0.5).float()}
    cfg = {"device": "cuda", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1, "loss": "bce_dice",
           "precision": "fp32", "max_grad_norm": 1.0}
    torch.manual_seed(0)
    tr = Trainer(cfg)
    l0 = tr.step(batch)
    torch.manual_seed(0)
    from pcms_amd.models.unet3d import UNet3D
    m = UNet3D(n_modalities=5, n_classes=1, precision="fp32").cuda()
    opt = FlatAdam(m, lr=1e-4, weight_decay=1e-5)
    opt.zero_grad()
    loss = BCEDiceLoss()(m(batch["image"].cuda()), batch["label"].cuda())
    loss.backward()
    norm = clip_grad_norm_(m, 1.0)
    opt.step()
    assert float(loss) == l0
    assert float(norm) > 1.0  # the clip engaged at init
    assert float(tr.last_grad_norm) == pytest.approx(float(norm), rel=1e-6)
    for (k, a), b in zip(tr.model.named_parameters(), m.parameters()):
        torch.testing.assert_close(a, b, rtol=0, atol=1e-7, msg=k)
        torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-12, msg=k)


@pytest.mark.gpu
def test_grad_scaler_step_skip_and_scale_update():
    from pcms_amd.amp import GradScaler
    from pcms_amd.utils.trainer import Trainer
    gen = torch.Generator().manual_seed(9)
    batch = {"image": torch.rand(2, 5, 16, 16, 16, generator=gen),
             "label": (torch.rand(2, 1, 16, 16, 16, generator=gen) < 0.5).float()}
    base = {"device": "cuda", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1, "loss": "bce_dice",
            "precision": "bf16"}
    torch.manual_seed(0)
    plain = Trainer(base)
    torch.manual_seed(0)
    amp = Trainer(dict(base, use_amp=True))
    assert isinstance(amp.scaler, GradScaler) and amp.scaler.get_scale() == 2.0 ** 16
    l_plain, l_amp = plain.step(batch), amp.step(batch)
    assert l_plain == l_amp  # the returned loss is the unscaled one
    # a power-of-two loss scale unscales exactly: same update as the unscaled step, up to
    # the bf16 rounding of the scaled activation gradients
    for (k, a), b in zip(plain.model.named_parameters(), amp.model.parameters()):
        assert torch.allclose(a, b, rtol=0, atol=2.01e-4), k
    assert amp.scaler.get_scale() == 2.0 ** 16
    # an inf gradient: the step is skipped, the scale backs off
    p_before = amp.model.engine().flat_p.clone()
    sc = amp.scaler
    eng = amp.model.engine()
    amp.optimizer.zero_grad(set_to_none=False)  # grads stay attached (zeroed), as after a backward
    eng.flat_g[123] = float("inf")
    sc.unscale_(amp.optimizer)
    sc.step(amp.optimizer)
    sc.update()
    assert torch.equal(eng.flat_p, p_before)
    assert sc.get_scale() == 2.0 ** 15
    # growth after growth_interval clean steps
    sc.growth_interval = 2
    for _ in range(2):
        amp.step(batch)
    assert sc.get_scale() == 2.0 ** 16
    assert math.isfinite(float(amp.last_grad_norm))


@pytest.mark.gpu
@pytest.mark.parametrize("gscale", [1.0, 0.5])
@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_fused_adam_packs_match_flat_adam(gscale, precision):
    """The fused Adam (pcms_adam_pack_conv3 / _convt / _ranges, engine.adam_plan; the fp32
    build's _x6 forms write the bf16x6 packs) matches the flat Adam kernel (same per-element
    arithmetic; the compiler may contract it differently, so to 1e-6 relative), and the conv /
    ConvT weight packs it writes are bit-identical to the pack kernels run on the updated
    master."""
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    gen = torch.Generator().manual_seed(2)
    x = torch.rand(2, 5, 16, 16, 16, generator=gen).cuda()
    y = (torch.rand(2, 1, 16, 16, 16, generator=gen) < 0.5).float().cuda()
    runs = []
    for fused in (False, True):
        torch.manual_seed(0)
        m = UNet3D(n_modalities=5, n_classes=1, precision=precision).cuda()
        opt = FlatAdam(m, lr=1e-3, weight_decay=1e-5)
        opt.fused_packs = fused
        opt.zero_grad()
        BCEDiceLoss()(m(x), y).backward()
        opt.grad_scale = gscale
        opt.step()
        eng = m.engine()
        eng._ensure_packs()
        eng._stem_conv_pack()  # the stem's general-kernel pack is otherwise built on first use
        torch.cuda.synchronize()
        runs.append((eng, opt))
    (e0, o0), (e1, o1) = runs
    plan = e1.adam_plan()
    assert plan["nconv"] == 17 and plan["nconvt"] == 4 and plan["complete"]
    assert plan["x6"] == (precision == "fp32")
    for a, b in ((e0.flat_p, e1.flat_p), (e0.flat_g, e1.flat_g), (o0._m, o1._m), (o0._v, o1._v)):
        torch.testing.assert_close(b, a, rtol=1e-6, atol=1e-12)
    # (the general kernel's packs of convs that run only on the 16x16x32 kernel are skipped
    # by the fused Adam and rebuilt on use: test_fused_adam_writes_pack16)
    packs = [(t, t.clone()) for cs in e1.convs if not cs.old_stale for t in (cs.fwd, cs.dgrad) if t is not None]
    packs += [(t, t.clone()) for i in range(4) for t in e1.convt_packs[i]]
    packs += [(t, t.clone()) for cs in e1.convs for t in (cs.fwd16, cs.dgrad16) if t is not None]
    assert len(packs) >= 21
    e1.mark_dirty()
    e1._ensure_packs()  # full repack from the fused step's master (in place)
    torch.cuda.synchronize()
    for t, a in packs:
        assert torch.equal(a.view(torch.int16), t.view(torch.int16))


@pytest.mark.gpu
def test_fused_adam_writes_pack16():
    """At a shape where the 16x16x32 kernel runs (1 x 5x128x128x64), the fused Adam also writes
    the pack16 forms (no separate pcms_conv3_pack16 pass) and skips the general kernel's packs
    of the convs no call used; both are bit-identical to the pack kernels run on the updated
    master, and a skipped pack is rebuilt on first use (engine._old_packs), which re-plans."""
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    gen = torch.Generator().manual_seed(3)
    x = torch.rand(1, 5, 128, 128, 64, generator=gen).cuda()
    y = (torch.rand(1, 1, 128, 128, 64, generator=gen) < 0.5).float().cuda()
    torch.manual_seed(0)
    m = UNet3D(n_modalities=5, n_classes=1, precision="bf16").cuda()
    opt = FlatAdam(m, lr=1e-3, weight_decay=1e-5)
    for _ in range(2):
        opt.zero_grad()
        BCEDiceLoss()(m(x), y).backward()
        opt.step()
    eng = m.engine()
    plan = eng._adam_plan
    assert plan is not None and plan["p16"] and plan["complete"]
    with16 = [cs for cs in eng.convs if cs.fwd16 is not None or cs.dgrad16 is not None]
    assert len(with16) >= 8
    assert plan["old_skip"] and all(cs.old_stale for cs in plan["old_skip"])
    p16 = [t.clone() for cs in with16 for t in (cs.fwd16, cs.dgrad16) if t is not None]
    old = {id(cs): (cs.fwd.clone(), cs.dgrad.clone()) for cs in eng.convs[1:] if not cs.old_stale}
    # a skipped pack, rebuilt on use
    cs = plan["old_skip"][0]
    eng._old_packs(cs)
    assert not cs.old_stale and cs.old_used and eng._adam_plan is None
    lazy = (cs.fwd.clone(), cs.dgrad.clone())
    eng.mark_dirty()
    eng._ensure_packs()  # full repack (general packs + pcms_conv3_pack16) from the same master
    torch.cuda.synchronize()
    fresh = [t for c in with16 for t in (c.fwd16, c.dgrad16) if t is not None]
    for a, b in zip(p16, fresh):
        assert torch.equal(a.view(torch.int16), b.view(torch.int16))
    for c in eng.convs[1:]:
        if id(c) in old:
            assert torch.equal(old[id(c)][0].view(torch.int16), c.fwd.view(torch.int16))
            assert torch.equal(old[id(c)][1].view(torch.int16), c.dgrad.view(torch.int16))
    assert torch.equal(lazy[0].view(torch.int16), cs.fwd.view(torch.int16))
    assert torch.equal(lazy[1].view(torch.int16), cs.dgrad.view(torch.int16))


def _oracle_amp_clip_step(x, y, max_norm, init_scale=2.0 ** 16):
    """The reference's mixed-precision step with the clip of its other trainers, on the CPU
    oracle with torch's own GradScaler (train_bph_optimized.py:296-298 + train_bph.py:166):
    scaler.scale(loss).backward(); scaler.unscale_(opt); clip_grad_norm_(params, max_norm);
    scaler.step(opt); scaler.update()."""
    from oracle import unet3d_cpu as ref
    from tests import golden_util as gu
    torch.manual_seed(0)
    sd = ref.init_params(5, 1)
    keys = ref.param_keys(sd)
    p0 = {k: sd[k].detach().clone() for k in keys}
    for k in keys:
        sd[k].requires_grad_(True)
    params = [sd[k] for k in keys]
    opt = torch.optim.Adam(params, lr=1e-4, weight_decay=1e-5)
    scaler = torch.amp.GradScaler("cpu", init_scale=init_scale)
    loss = ref.bce_dice_loss(ref.forward(sd, x, training=True), y)
    scaler.scale(loss).backward()
    scaler.unscale_(opt)
    norm = float(torch.nn.utils.clip_grad_norm_(params, max_norm))
    grads = {k: sd[k].grad.detach().clone() for k in keys}
    scaler.step(opt)
    scaler.update()
    # the fp64 truth of the unclipped gradient norm (at 16^3 the bottleneck BatchNorm sees 2
    # values per channel: two fp32 runs' norms differ by ~1e-3 relative)
    torch.manual_seed(0)
    g64 = gu.oracle_grads64(ref.init_params(5, 1), x, y)
    norm64 = float(torch.sqrt(sum((g.double() ** 2).sum() for g in g64.values())))
    clip64 = min(1.0, max_norm / (norm64 + 1e-6))
    return {"loss": float(loss), "norm": norm, "norm64": norm64, "grads": grads, "p0": p0,
            "grads64": {k: g * clip64 for k, g in g64.items()},
            "post": {k: v.detach().clone() for k, v in sd.items()}, "scale": scaler.get_scale()}


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["user_sequence", "trainer"])
def test_amp_clip_step_matches_oracle_torch_gradscaler(path):
    """AMP + clip against the oracle driven by torch.amp.GradScaler (not against our own
    engine): ``user_sequence`` is torch's documented unscale_ -> clip_grad_norm_ -> step
    pattern on our GradScaler / clip (unscale_ must leave unscaled gradients in
    param.grad); ``trainer`` is Trainer(use_amp, max_grad_norm).step with unscale and clip
    folded into the Adam pass.  Same loss, same total norm, gradients (left in param.grad:
    unscaled and clipped) within the 16^3 golden bar, post-step parameters with the
    confident-element bar (tests/golden_util.check_step_against_oracle)."""
    from pcms_amd.amp import GradScaler, clip_grad_norm_
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    from pcms_amd.utils.trainer import Trainer
    from tests import golden_util as gu
    gen = torch.Generator().manual_seed(9)
    x = torch.rand(2, 5, 16, 16, 16, generator=gen)
    y = (torch.rand(2, 1, 16, 16, 16, generator=gen) < 0.5).float()
    r = _oracle_amp_clip_step(x, y, 1.0)
    torch.manual_seed(0)
    if path == "user_sequence":
        m = UNet3D(n_modalities=5, n_classes=1, precision="fp32").cuda()
        opt = FlatAdam(m, lr=1e-4, weight_decay=1e-5)
        sc = GradScaler()
        opt.zero_grad()
        loss = BCEDiceLoss()(m(x.cuda()), y.cuda())
        sc.scale(loss).backward()
        sc.unscale_(opt)
        # param.grad now holds the unscaled gradient (torch semantics)
        g_unscaled = torch.cat([p.grad.detach().reshape(-1) for p in m.parameters()]).double()
        norm = float(clip_grad_norm_(m, 1.0, opt))
        assert abs(float(g_unscaled.norm()) - norm) <= 1e-6 * norm
        sc.step(opt)
        sc.update()
        loss = float(loss)
        scale = sc.get_scale()
    else:
        tr = Trainer({"device": "cuda", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1,
                      "loss": "bce_dice", "precision": "fp32", "use_amp": True, "max_grad_norm": 1.0})
        m = tr.model
        loss = tr.step({"image": x, "label": y})
        norm = float(tr.last_grad_norm)
        scale = tr.scaler.get_scale()
    torch.cuda.synchronize()
    assert abs(loss - r["loss"]) <= 1e-5, (loss, r["loss"])
    n64 = r["norm64"]
    assert abs(norm - n64) <= max(10 * abs(r["norm"] - n64), 1e-3 * n64), (norm, r["norm"], n64)
    assert norm > 1.0  # the clip engaged
    assert scale == r["scale"]
    grads = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}
    gu.check_step_against_oracle(m, grads, r, grad_rl2=5e-2, min_confident=0.2)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_fresh_gradient_store_equals_zero_fill(precision):
    """zero_grad() (set_to_none, torch's default) leaves param.grad None and the next backward
    WRITES the conv weight gradients (PCMS_GRAD_STORE) after zeroing only the other ranges;
    zero_grad(set_to_none=False) zero-fills and the backward accumulates.  Both give the same
    gradient bit for bit; a second backward without zero_grad accumulates (sum of both)."""
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    gen = torch.Generator().manual_seed(3)
    x = torch.rand(2, 5, 32, 32, 16, generator=gen).cuda()
    y = (torch.rand(2, 1, 32, 32, 16, generator=gen) < 0.4).float().cuda()
    torch.manual_seed(0)
    m = UNet3D(n_modalities=5, n_classes=1, precision=precision).cuda()
    opt = FlatAdam(m, lr=1e-3, weight_decay=1e-5)
    eng = m.engine()
    eng.flat_g.fill_(float("nan"))  # stale contents must not leak into a fresh gradient
    opt.zero_grad()
    assert all(p.grad is None for p in m.parameters())
    BCEDiceLoss()(m(x), y).backward()
    assert eng._gstore
    g_store = eng.flat_g.clone()
    assert torch.isfinite(g_store).all()
    opt.zero_grad(set_to_none=False)
    BCEDiceLoss()(m(x), y).backward()
    assert not eng._gstore
    assert torch.equal(eng.flat_g, g_store)
    BCEDiceLoss()(m(x), y).backward()  # accumulates
    torch.testing.assert_close(eng.flat_g, 2 * g_store, rtol=1e-6, atol=0)
    assert all(p.grad is not None and p.grad.data_ptr() >= eng.flat_g.data_ptr() for p in m.parameters())


@pytest.mark.gpu
def test_bnin_fusion_step_bit_identical():
    """A whole bf16 training step with the DoubleConvs' first BatchNorm + ReLU fused into the
    second conv's staging (engine.fuse_bnin, forward and weight gradient) equals the step with
    the separate a1 = relu(bn(y1)) pass bit for bit: logits, loss, every gradient, the Adam
    update and the BatchNorm buffers (level 0: 2 x 64x64x32, the fused kernels' smallest
    unsplit big-box size)."""
    from pcms_amd import _lib as L
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    gen = torch.Generator().manual_seed(8)
    x = torch.rand(2, 5, 64, 64, 32, generator=gen).cuda()
    y = (torch.rand(2, 1, 64, 64, 32, generator=gen) < 0.4).float().cuda()
    old = L.query("pcms_conv3_big_min_boxes", -1)
    try:
        runs = []
        for fuse in (False, True):
            torch.manual_seed(0)
            m = UNet3D(n_modalities=5, n_classes=1).cuda()
            eng = m.engine()
            eng.fuse_bnin = fuse
            opt = FlatAdam(m, lr=1e-3, weight_decay=1e-5)
            opt.zero_grad()
            lg = m(x)
            loss = BCEDiceLoss()(lg, y)
            loss.backward()
            g = eng.flat_g.clone()
            opt.step()
            torch.cuda.synchronize()
            if fuse:
                assert eng._bnin(eng.enc[0], 2, (64, 64, 32)), "the fused kernels did not run"
            runs.append((lg.detach().clone(), float(loss.detach()), g, eng.flat_p.clone(), eng.flat_bn.clone()))
        (l0, s0, g0, p0, b0), (l1, s1, g1, p1, b1) = runs
        assert torch.equal(l0, l1) and s0 == s1
        assert torch.equal(g0, g1)
        assert torch.equal(p0, p1)
        assert torch.equal(b0, b1)
    finally:
        L.query("pcms_conv3_big_min_boxes", old)


@pytest.mark.gpu
@pytest.mark.parametrize("ckpt", [False, True])
def test_convt_wgrad_side_step_bit_identical(ckpt):
    """The ConvTranspose weight + bias gradients on the side stream beside the ConvT dgrad
    (engine.convt_wgrad_side, their own partial-row workspace) give the same two bf16 training
    steps bit for bit as the serial order: logits, losses, every gradient, the Adam updates and
    the BatchNorm buffers (2 x 64x64x32; with and without decoder checkpointing, whose recompute
    joins the side stream first)."""
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    gen = torch.Generator().manual_seed(9)
    x = torch.rand(2, 5, 64, 64, 32, generator=gen).cuda()
    y = (torch.rand(2, 1, 64, 64, 32, generator=gen) < 0.4).float().cuda()
    runs = []
    for side in (False, True):
        torch.manual_seed(0)
        m = UNet3D(n_modalities=5, n_classes=1, checkpoint_decoder=ckpt).cuda()
        eng = m.engine()
        eng.convt_wgrad_side = side
        opt = FlatAdam(m, lr=1e-3, weight_decay=1e-5)
        out = []
        for _ in range(2):
            opt.zero_grad()
            lg = m(x)
            loss = BCEDiceLoss()(lg, y)
            loss.backward()
            g = eng.flat_g.clone()
            opt.step()
            out += [lg.detach().clone(), loss.detach().clone(), g]
        torch.cuda.synchronize()
        assert ("ctws_w" in eng.bufs) == side
        runs.append(out + [eng.flat_p.clone(), eng.flat_bn.clone()])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "fp32"])
@pytest.mark.parametrize("S", [(64, 64, 32), (20, 18, 24)])
def test_pool_bn_apply_fused_step_bit_identical(precision, S):
    """The encoder's MaxPool3d backward writing only the BN-backward partial rows
    (pcms_maxpool_bwd_bn_sums) with the pooled gradient added again inside that BatchNorm's
    apply (pcms_maxpool_bn_apply, engine.pool_bn_apply_fused) gives the same two training steps
    bit for bit as pcms_maxpool_bwd_bn + pcms_bn_relu_bwd_finish: logits, losses, every
    gradient, the Adam updates and the BatchNorm buffers -- at an even size and at one whose
    odd levels leave floor-mode leftovers (partial 2x2x2 cells)."""
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    gen = torch.Generator().manual_seed(10)
    x = torch.rand(2, 5, *S, generator=gen).cuda()
    y = (torch.rand(2, 1, *S, generator=gen) < 0.4).float().cuda()
    runs = []
    for fused in (False, True):
        torch.manual_seed(0)
        m = UNet3D(n_modalities=5, n_classes=1, precision=precision).cuda()
        eng = m.engine()
        eng.pool_bn_apply_fused = fused
        opt = FlatAdam(m, lr=1e-3, weight_decay=1e-5)
        out = []
        for _ in range(2):
            opt.zero_grad()
            lg = m(x)
            loss = BCEDiceLoss()(lg, y)
            loss.backward()
            out += [lg.detach().clone(), loss.detach().clone(), eng.flat_g.clone()]
            opt.step()
        torch.cuda.synchronize()
        runs.append(out + [eng.flat_p.clone(), eng.flat_bn.clone()])
    for a, b in zip(*runs):
        assert torch.equal(a, b)
