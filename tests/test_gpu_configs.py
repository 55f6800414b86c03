"""The single-GPU BASELINE.json configs at their full sizes, on MI355X.

* config 2: UNet3D 5->1, 2 x 5x128x128x64, BCEDiceLoss.
* config 4: the same with zero_fill missing modalities (1-2 of 5 channels all-zero per
  sample, script/data_loader.py:320-322).
* config 5: 1 x 5x256x256x96 with decoder activation checkpointing.

Pinned to the REFERENCE itself: tests/golden/full_<cfg>.npz were written by
tests/golden/make_golden_full.py, which runs the reference's own models/unet3d.py UNet3D and
utils/losses.py BCEDiceLoss (one step of utils/trainer.py:183-192, fp32; the same forward +
backward in fp64 for configs 2 / 4 and under CPU bf16 autocast) on the same seed-0 init and
seed-1234 batch (pins: tests/test_oracle_golden.py::test_full_fixtures_pinned).  No oracle runs
on the GPU box's host.  Bars:
* fp32 build, configs 2 and 4, a whole training step: train-mode logits within 1e-3 (at the
  fixture's 2^18 sampled positions), identical ``logit > 0`` masks where |ref| >= 1e-3 (every
  voxel), loss within 1e-5; every gradient's relative L2 distance to the reference's fp64
  gradient within max(5e-3, 10x the reference's fp32 distance to it) (the 18 pre-BN conv
  biases, exact gradient 0, within 1e-4 absolute); the post-Adam parameters within
  2.01 lr everywhere and within 1e-5 relative on "confident" elements; BatchNorm running
  statistics within 1e-4 relative (gradients / parameters at 8192 strided positions per tensor).
* bf16 build (bf16 storage cannot meet 1e-3): against the reference's fp32 run with
  a bar set by the reference's bf16-autocast run: max |dlogit| <= 2x the autocast run's (same
  sampled positions), mask agreement >= the autocast run's - 0.5 % (every voxel), loss within
  2x the autocast run's loss error (floor 1e-3).  Configs 2, 4 and 5 (config 5: the
  decoder-checkpointed step, and every gradient within max(3x the autocast run's relative L2
  distance to the fp32 gradient, 2e-2)).
* Dense windows (configs 2 and 4): besides the strided 2^18-position sample, every logit of the
  volume faces and of the planes either side of the 8-voxel (d, h) / 16-voxel (w) box seams
  (win_axis / win_index / w32__ / wbf__ in the fixture): fp32 within 1e-3, bf16 within 2x the
  autocast run's largest error on the same planes.

The autocast bar is not the reference's single-call arithmetic everywhere: oneDNN's CPU bf16
conv backward faults past ~2^28 elements per call, so make_golden_full.py ran the layers the
fixture's ``autocast_chunked`` lists (the level-0 convs at configs 2 / 4; those plus up3.conv.0
and up4.up at config 5) over d-slabs, each slab casting its own operands (the same bf16 sums per
output, slab partials of the weight gradients added in fp32).  Config 5's bf16 gradient bar
comes only from such a run (no fp32 truth at that size): parity unpinned there in the strict
sense, pinned to a slab-chunked autocast run of the reference's modules.
"""
import pytest
import torch

from tests import golden_util as gu

pytestmark = pytest.mark.gpu

CFG2 = (2, (128, 128, 64))
CFG5 = (1, (256, 256, 96))


@pytest.fixture(scope="module", params=["cfg2", "cfg4"], ids=["cfg2", "cfg4_zero_fill"])
def fixture_run(request):
    """The reference's step at config 2 / 4 (the committed fixture) and the batch it ran on."""
    cfg = request.param
    fx = gu.full_fixture(cfg)
    x, y = gu.full_batch(cfg)
    assert abs(float(x.double().sum()) - float(fx["input_sum"])) <= 1e-6 * abs(float(fx["input_sum"]))
    if cfg == "cfg4":
        per_sample_zero = (x.abs().amax(dim=(2, 3, 4)) == 0).sum(1)
        assert all(1 <= int(k) <= 2 for k in per_sample_zero)
    return {"cfg": cfg, "fx": fx, "x": x, "y": y}


def _gpu_step(precision, x, y, ckpt=False, keep_grad=False, keep_p0=False):
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss
    torch.manual_seed(0)
    m = UNet3D(n_modalities=5, n_classes=1, precision=precision, checkpoint_decoder=ckpt).cuda()
    p0 = {k: p.detach().cpu().clone() for k, p in m.named_parameters()} if keep_p0 else None
    opt = FlatAdam(m, lr=1e-4, weight_decay=1e-5)
    crit = BCEDiceLoss()
    m.train()
    opt.zero_grad()
    logits = m(x.cuda())
    loss = crit(logits, y.cuda())
    loss.backward()
    grads = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()} if keep_grad else None
    opt.step()
    torch.cuda.synchronize()
    if keep_p0:
        return m, logits.detach().cpu(), float(loss.detach()), grads, p0
    if keep_grad:
        return m, logits.detach().cpu(), float(loss.detach()), grads
    return m, logits.detach().cpu(), float(loss.detach())


def _logits_vs_fixture(lg, fx):
    st = int(fx["logit_stride"])
    return lg.reshape(-1)[::st].double(), torch.from_numpy(fx["l32_s"]).double(), torch.from_numpy(fx["lbf_s"]).double()


def test_fp32_build_matches_reference(fixture_run):
    r = fixture_run
    fx = r["fx"]
    m, lg, loss, grads, p0 = _gpu_step("fp32", r["x"], r["y"], keep_grad=True, keep_p0=True)
    got, ref, _ = _logits_vs_fixture(lg, fx)
    err = (got - ref).abs().max().item()
    assert err <= 1e-3, err
    n = lg.numel()
    sure = gu.unpack_bits(fx["sure_bits"], n)
    m32 = gu.unpack_bits(fx["m32_bits"], n)
    mine = (lg > 0).reshape(-1)
    assert torch.equal(mine[sure], m32[sure])
    assert abs(loss - float(fx["loss32"])) <= 1e-5, (loss, float(fx["loss32"]))
    werr = _window_errors(lg, fx)
    if werr is not None:
        assert werr <= 1e-3, werr
    rep = {}
    params = {k: p.detach().cpu() for k, p in m.named_parameters()}
    gu.check_step_against_fixture(params, grads, p0, m.state_dict(), fx, report=rep)
    print(f"\n[{r['cfg']} fp32 vs reference] max|dlogit| {err:.2e} (dense windows {werr}), worst grad rel-L2 "
          f"{rep['worst_grad_rl2'][0]:.2e} ({rep['worst_grad_rl2'][1]}), confident params {rep['confident']:.3f}")
    gu.record_margin(f"{r['cfg']}_fp32", max_dlogit=err, logit_bar=1e-3, window_max_dlogit=werr,
                     loss_err=abs(loss - float(fx["loss32"])), loss_bar=1e-5, worst_grad=rep["worst_grad_rl2"],
                     worst_grad_over_bar=rep["worst_grad_over_bar"], confident=rep["confident"],
                     masks_equal_where_sure=True)


def _window_errors(lg, fx, tag="build"):
    """max |logit - reference fp32 logit| over the fixture's dense planes: of the GPU logits
    ``lg`` (tag "build") or of the reference's own autocast run (tag "bf"); None for a fixture
    without planes."""
    if "win_axis" not in fx:
        return None
    err = 0.0
    for i, (ax, j) in enumerate(zip(fx["win_axis"], fx["win_index"])):
        base = torch.from_numpy(fx[f"w32__{i}"]).double()
        got = (lg.select(int(ax), int(j)).reshape(-1).double() if tag == "build"
               else torch.from_numpy(fx[f"w{tag}__{i}"]).double())
        err = max(err, float((got - base).abs().max()))
    return err


def test_bf16_build_within_bf16_bar(fixture_run):
    r = fixture_run
    _, lg, loss = _gpu_step("bf16", r["x"], r["y"])
    marg = _bf16_bar(lg, loss, r["fx"], r["cfg"])
    fx = r["fx"]
    werr = _window_errors(lg, fx)
    if werr is not None:
        wauto = _window_errors(None, fx, "bf")
        print(f"[{r['cfg']} bf16] dense windows max|dlogit| {werr:.4f} (autocast {wauto:.4f})")
        assert werr <= 2 * wauto, (werr, wauto)
        marg.update(window_max_dlogit=werr, window_autocast=wauto)
    gu.record_margin(f"{r['cfg']}_bf16", **marg)


def test_config2_full_step_deterministic():
    """Two full bf16 steps at config 2 from the same init and batch are bit-identical."""
    from pcms_amd.synthetic import make_batch
    b = make_batch(*CFG2, seed=1234)
    outs = []
    for _ in range(2):
        m, lg, loss = _gpu_step("bf16", b["image"], b["label"])
        outs.append((lg, loss, m.engine().flat_g.detach().clone(), m.engine().flat_p.detach().clone()))
        del m
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]
    assert torch.equal(outs[0][2], outs[1][2])
    assert torch.equal(outs[0][3], outs[1][3])


def test_config5_checkpointed_vs_plain():
    """Config 5 (1 x 5x256x256x96): the checkpointed step equals the plain one bit for bit
    (loss, every gradient, the Adam update) and BatchNorm counts exactly one update per step."""
    from pcms_amd.synthetic import make_batch
    b = make_batch(*CFG5, seed=1234)
    res = []
    for ckpt in (False, True):
        m, lg, loss = _gpu_step("bf16", b["image"], b["label"], ckpt=ckpt)
        nbt = [int(v) for k, v in m.state_dict().items() if k.endswith("num_batches_tracked")]
        res.append((loss, m.engine().flat_g.detach().clone(), m.engine().flat_p.detach().clone(),
                    m.engine().flat_bn.detach().clone(), nbt))
        del m
        torch.cuda.empty_cache()
    (l0, g0, p0, b0, n0), (l1, g1, p1, b1, n1) = res
    assert l0 == l1
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)
    assert torch.equal(b0, b1)
    assert n0 == n1 == [1] * 18


def _bf16_bar(lg, loss, fx, tag):
    got, ref, auto = _logits_vs_fixture(lg, fx)
    e_auto = (auto - ref).abs().max().item()
    e = (got - ref).abs().max().item()
    n = lg.numel()
    m32 = gu.unpack_bits(fx["m32_bits"], n)
    agree_auto = float(fx["agree_auto"])
    agree = ((lg > 0).reshape(-1) == m32).float().mean().item()
    loss32, lossbf = float(fx["loss32"]), float(fx["lossbf"])
    print(f"\n[{tag} bf16 vs reference] max|dlogit| {e:.4f} (autocast {e_auto:.4f}; full tensor "
          f"{float(fx['e_auto']):.4f}), masks {agree:.5f} (autocast {agree_auto:.5f}), "
          f"loss {loss:.6f} vs {loss32:.6f} (autocast {lossbf:.6f})")
    assert e <= 2 * e_auto, (e, e_auto)
    assert agree >= agree_auto - 0.005, (agree, agree_auto)
    assert abs(loss - loss32) <= max(2 * abs(lossbf - loss32), 1e-3), (loss, loss32, lossbf)
    return {"max_dlogit": e, "autocast_max_dlogit": e_auto, "dlogit_over_bar": e / (2 * e_auto),
            "mask_agree": agree, "autocast_mask_agree": agree_auto, "loss_err": abs(loss - loss32),
            "loss_bar": max(2 * abs(lossbf - loss32), 1e-3),
            "autocast_chunked": [str(v) for v in fx["autocast_chunked"]] if "autocast_chunked" in fx else None}


def test_config5_checkpointed_bf16_vs_reference():
    """Config 5 (1 x 5x256x256x96, decoder checkpointing, bf16) against the reference's step at
    that shape (tests/golden/full_cfg5.npz) with the autocast-relative bf16 bar (train logits /
    masks / loss as at configs 2 and 4), and every gradient: its relative L2 distance to the
    reference's fp32 gradient within max(3x the reference's bf16-autocast run's distance, 2e-2),
    on the fixture's sample positions (pre-BN conv biases, exact gradient 0, SURVEY H5: within
    1e-4 absolute).  Parity unpinned in the strict sense: the autocast run that sets the bar is
    slab-chunked at the six layers ``autocast_chunked`` lists (module docstring)."""
    fx = gu.full_fixture("cfg5")
    x, y = gu.full_batch("cfg5")
    assert abs(float(x.double().sum()) - float(fx["input_sum"])) <= 1e-6 * abs(float(fx["input_sum"]))
    m, lg, loss, grads = _gpu_step("bf16", x, y, ckpt=True, keep_grad=True)
    del m
    torch.cuda.empty_cache()
    marg = _bf16_bar(lg, loss, fx, "cfg5 ckpt")
    worst = (0.0, "")
    rows = []
    for k, g in grads.items():
        got = gu.fixture_sampled(g, fx, k)
        if k.endswith(gu.PRE_BN_BIAS):
            assert got.abs().max() < 1e-4, k
            continue
        t = torch.from_numpy(fx["g32__" + k]).double()
        nrm = max(float(t.norm()), 1e-30)
        rl = float((got - t).norm()) / nrm
        rl_auto = float((torch.from_numpy(fx["gbf__" + k]).double() - t).norm()) / nrm
        bar = max(3 * rl_auto, 2e-2)
        rows.append((k, rl, rl_auto))
        worst = max(worst, (rl / bar, k))
    for k, rl, rl_auto in rows:
        print(f"  {k:48s} rel-L2 {rl:.3e} (reference autocast {rl_auto:.3e})")
    print(f"[cfg5 ckpt bf16 vs reference] worst gradient rel-L2 / bar {worst[0]:.3f} ({worst[1]})")
    gu.record_margin("cfg5_ckpt_bf16", worst_grad_over_bar=worst, **marg)
    for k, rl, rl_auto in rows:
        assert rl <= max(3 * rl_auto, 2e-2), (k, rl, rl_auto)
