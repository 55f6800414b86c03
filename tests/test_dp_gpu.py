"""The real data-parallel Trainer.step on the GPU: two ranks, one process each,
sharing cuda:0 over gloo with CUDA tensors (RCCL needs one GPU per rank; the 8-GPU RCCL run
is the driver's).  It runs every piece of utils/trainer.py's distributed branch: rank-0
BatchNorm-buffer broadcast, the engine's module-completion hook driving the bucketed
all-reduce beside the backward, the 1/world mean folded into Adam, optionally the fused
gradient clip.  Checked against ``oracle.dp_step_simulated`` (DDP broadcast_buffers
semantics around the reference step, utils/trainer.py:183-192): per-replica losses, the mean
gradient left in param.grad, BatchNorm buffers = rank 0's, Adam-step parameters."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from tests import golden_util as gu

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PRE_BN_BIAS = ("conv.0.bias", "conv.3.bias")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, world, clip=0.0, spatial="32,32,16", precision="fp32", ckpt=False, tag="dp"):
    out = str(tmp_path / f"{tag}.pt")
    port = str(_port())
    env = dict(os.environ, CLIP=str(clip), PCMS_DP_STEPS="1", PCMS_DP_SPATIAL=spatial, PCMS_DP_PRECISION=precision,
               PCMS_DP_CKPT="1" if ckpt else "0")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "tools", "dp_worker.py"), str(r), str(world), port,
                               out], env=env) for r in range(world)]
    rcs = [p.wait(timeout=240) for p in procs]
    assert rcs == [0] * world, rcs
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("clip", [0.0, 1.0])
def test_dp_trainer_step_two_ranks(tmp_path, clip):
    from oracle import unet3d_cpu as ref
    from pcms_amd.synthetic import make_batch, step_seed
    world = 2
    r = _run(tmp_path, world, clip)
    torch.manual_seed(0)
    sd = ref.init_params(5, 1)
    keys = ref.param_keys(sd)
    shards = []
    for rk in range(world):
        b = make_batch(2, (32, 32, 16), seed=step_seed(rk, 0), label="bernoulli")
        shards.append((b["image"], b["label"]))
    # the simulation's replica losses and mean gradient, computed the way dp_step_simulated does
    losses, grads = [], None
    for img, lab in shards:
        rep = {k: v.detach().clone() for k, v in sd.items()}
        for k in keys:
            rep[k].requires_grad_(True)
        l = ref.bce_dice_loss(ref.forward(rep, img, training=True), lab)
        l.backward()
        losses.append(float(l))
        g = torch.cat([rep[k].grad.reshape(-1) for k in keys])
        grads = g if grads is None else grads + g
    mean_g = grads / world
    # the fp64 truth of the mean gradient (the bar of the golden tests: within 10x the fp32
    # oracle's own distance to it, or 5e-3 relative L2)
    g64 = None
    for img, lab in shards:
        gg = gu.oracle_grads64(sd, img, lab)
        gv = torch.cat([gg[k].reshape(-1) for k in keys])
        g64 = gv if g64 is None else g64 + gv
    mean_g64 = g64 / world
    for rk in range(world):
        assert abs(r["losses"][rk][0] - losses[rk]) <= 1e-5, (rk, r["losses"][rk][0], losses[rk])
    norm = float(mean_g.double().norm())
    coef = min(1.0, clip / (norm + 1e-6)) if clip > 0 else 1.0
    if clip > 0:
        assert abs(r["norm"] - norm) <= 1e-3 * norm, (r["norm"], norm)
        assert coef < 1.0  # the clip engaged
    # param.grad holds the DDP mean (x the clip coefficient) after optimizer.step()
    off = 0
    for k in keys:
        n = sd[k].numel()
        got, exp = r["grad"][off:off + n].double(), (mean_g[off:off + n] * coef).double()
        off += n
        if k.endswith(PRE_BN_BIAS):
            assert got.abs().max() < 1e-4 * coef + 1e-12, k
            continue
        t = (mean_g64[off - n:off] * coef).double()
        nrm = float(t.norm().clamp_min(1e-30))
        rl = float((got - t).norm()) / nrm
        rl_ref = float((exp - t).norm()) / nrm
        assert rl <= max(5e-3, 10 * rl_ref), (k, rl, rl_ref)
    # Adam's first step moves each weight by ~lr * sign(g): within 2 lr of the simulation
    # everywhere, and within 1e-5 relative where the simulated |g + wd p| exceeds 8x the
    # tensor's largest gradient discrepancy (sign and size of the update fixed)
    p0 = {k: sd[k].detach().clone() for k in keys}
    _, _ = ref.dp_step_simulated(sd, shards, lr=1e-4, loss="bce_dice") if clip == 0 else (None, None)
    if clip == 0:
        off, nconf, ntot = 0, 0, 0
        for k in keys:
            n = sd[k].numel()
            got, exp = r["params"][off:off + n].double(), sd[k].detach().reshape(-1).double()
            gd = r["grad"][off:off + n].double()
            ge = mean_g[off:off + n].double()
            off += n
            d = (got - exp).abs()
            assert float(d.max()) <= 2.01e-4, (k, float(d.max()))
            if k.endswith(PRE_BN_BIAS):
                continue
            e = float((gd - ge).abs().max())
            conf = (ge + 1e-5 * p0[k].reshape(-1).double()).abs() > max(8 * e, 1e-6)
            nconf += int(conf.sum())
            ntot += n
            if conf.any():
                assert bool(torch.all(d[conf] <= 1e-5 * exp[conf].abs() + 2e-6)), (k, float(d[conf].max()))
        assert nconf >= 0.2 * ntot, (nconf, ntot)
        bn = torch.cat([sd[k].reshape(-1) for k in sd if k.endswith(("running_mean", "running_var"))])
        np.testing.assert_allclose(r["bn"].numpy(), bn.numpy(), rtol=1e-4, atol=1e-5)


def test_dp_trainer_step_config3_shape(tmp_path):
    """Config 3's per-rank workload (2 x 5x128x128x64 per rank, BASELINE configs[2]) through the
    real distributed Trainer.step (two ranks on cuda:0 over gloo, fp32 build, per-layer
    gradient readiness driving the bucketed all-reduce) against the REFERENCE's data-parallel
    step at that size (tests/golden/full_dp3.npz: the reference's UNet3D / BCEDiceLoss on each
    rank's shard, gradients averaged, one Adam step, rank 0's BatchNorm buffers; fp64 mean
    gradient as the truth).  Bars as the small two-rank test: per-replica losses within 1e-5,
    the mean gradient left in param.grad within max(5e-3, 10x the reference fp32 distance) of
    the fp64 mean (relative L2, at the fixture's sample positions; pre-BN conv biases < 1e-4),
    parameters within 2.01 lr and 1e-5 relative on confident elements, BatchNorm buffers =
    rank 0's."""
    import pcms_amd  # noqa: F401
    from pcms_amd.models.unet3d import UNet3D
    fx = gu.full_fixture("dp3")
    r = _run(tmp_path, 2, 0.0, "128,128,64")
    for rk in range(2):
        assert abs(r["losses"][rk][0] - float(fx["losses32"][rk])) <= 1e-5, (rk, r["losses"][rk][0])
    torch.manual_seed(0)
    m = UNet3D(n_modalities=5, n_classes=1)
    names = [k for k, _ in m.named_parameters()]
    params, grads, p0, off = {}, {}, {}, 0
    for k, p in m.named_parameters():
        n = p.numel()
        params[k] = r["params"][off:off + n]
        grads[k] = r["grad"][off:off + n]
        p0[k] = p.detach().reshape(-1)
        off += n
    bn_names = [k for k in m.state_dict() if k.endswith(("running_mean", "running_var"))]
    bufs, off = {}, 0
    for k in bn_names:
        n = m.state_dict()[k].numel()
        bufs[k] = r["bn"][off:off + n]
        off += n
    rep = {}
    gu.check_step_against_fixture(params, grads, p0, bufs, fx, report=rep, min_confident=0.2)
    print(f"\n[config-3 shape, 2 ranks] worst grad rel-L2 {rep['worst_grad_rl2'][0]:.2e} ({rep['worst_grad_rl2'][1]}), "
          f"confident params {rep['confident']:.3f}, {len(names)} tensors")
    gu.record_margin("dp3_fp32", loss_err=max(abs(r["losses"][rk][0] - float(fx["losses32"][rk])) for rk in range(2)),
                     loss_bar=1e-5, worst_grad=rep["worst_grad_rl2"], worst_grad_over_bar=rep.get("worst_grad_over_bar"),
                     confident=rep["confident"])


def _flat_views(r):
    """{name: flat tensor} of the parameters / gradients / BatchNorm buffers a worker saved,
    in the seed-0 model's order."""
    import pcms_amd  # noqa: F401
    from pcms_amd.models.unet3d import UNet3D
    torch.manual_seed(0)
    m = UNet3D(n_modalities=5, n_classes=1)
    params, grads, p0, off = {}, {}, {}, 0
    for k, p in m.named_parameters():
        n = p.numel()
        params[k], grads[k], p0[k] = r["params"][off:off + n], r["grad"][off:off + n], p.detach().reshape(-1)
        off += n
    bufs, off = {}, 0
    for k, v in m.state_dict().items():
        if k.endswith(("running_mean", "running_var")):
            bufs[k] = r["bn"][off:off + v.numel()]
            off += v.numel()
    return params, grads, p0, bufs


def test_dp_trainer_step_config3_shape_bf16(tmp_path):
    """BASELINE configs[2] at its product precision: the bf16 build through the real distributed
    Trainer.step (two ranks on cuda:0 over gloo, per-layer readiness driving the bucketed
    all-reduce, the bf16-only fused Adam pack writes and BN-input fusions) at config 3's
    per-rank workload (2 x 5x128x128x64 per rank), against the REFERENCE's two-rank step
    (tests/golden/full_dp3.npz, utils/trainer.py:183-192 per replica, gradients averaged, one
    Adam step, rank 0's buffers).  bf16 storage cannot meet the fp32 bars, so each
    bar is set by the reference's OWN CPU bf16-autocast run of the same two-rank step (lossesbf,
    gbf__, bbf__; slab-chunked at the layers ``autocast_chunked`` names, make_golden_full.py):
    * per-replica losses within max(2x the autocast loss error, 1e-3) of the fp32 losses;
    * the mean gradient left in param.grad: relative L2 distance to the reference's fp32 mean
      gradient within max(3x the autocast run's distance, 2e-2) per tensor (config 5's bar;
      pre-BN conv biases, exact gradient 0: within 1e-4 absolute);
    * rank 0's BatchNorm running statistics within 2x the autocast run's largest deviation from
      the fp32 buffers (+ 1e-5) per buffer, num_batches_tracked exact;
    * post-Adam parameters within 2.01 lr of the reference's everywhere (Adam's first step is
      ~lr sign(g))."""
    fx = gu.full_fixture("dp3")
    assert "lossesbf" in fx, "full_dp3.npz predates the autocast run (make_golden_full.py dp3bf)"
    r = _run(tmp_path, 2, 0.0, "128,128,64", precision="bf16", tag="dp3bf")
    loss_rows = []
    for rk in range(2):
        l32, lbf = float(fx["losses32"][rk]), float(fx["lossesbf"][rk])
        got = r["losses"][rk][0]
        bar = max(2 * abs(lbf - l32), 1e-3)
        loss_rows.append((abs(got - l32), bar))
        assert abs(got - l32) <= bar, (rk, got, l32, lbf)
    params, grads, p0, bufs = _flat_views(r)
    worst = (0.0, "")
    for k in params:
        got = gu.fixture_sampled(grads[k], fx, k)
        if k.endswith(PRE_BN_BIAS):
            assert got.abs().max() < 1e-4, k
            continue
        t = torch.from_numpy(fx["g32__" + k]).double()
        nrm = max(float(t.norm()), 1e-30)
        rl = float((got - t).norm()) / nrm
        rl_auto = float((torch.from_numpy(fx["gbf__" + k]).double() - t).norm()) / nrm
        bar = max(3 * rl_auto, 2e-2)
        worst = max(worst, (rl / bar, k))
        assert rl <= bar, (k, rl, rl_auto)
        d = (gu.fixture_sampled(params[k], fx, k) - torch.from_numpy(fx["post__" + k]).double()).abs()
        assert float(d.max()) <= 2.01e-4 + 1e-6, (k, float(d.max()))
    bworst = (0.0, "")
    for k, v in bufs.items():
        b32 = torch.from_numpy(fx["b__" + k]).double()
        dev_auto = float((torch.from_numpy(fx["bbf__" + k]).double() - b32).abs().max())
        dev = float((v.double() - b32).abs().max())
        bar = 2 * dev_auto + 1e-5
        bworst = max(bworst, (dev / bar, k))
        assert dev <= bar, (k, dev, dev_auto)
    print(f"\n[config-3 shape, 2 ranks, bf16] losses {[round(x[0], 6) for x in loss_rows]} (bars "
          f"{[round(x[1], 6) for x in loss_rows]}), worst grad rel-L2 / bar {worst[0]:.3f} ({worst[1]}), "
          f"worst BN buffer / bar {bworst[0]:.3f} ({bworst[1]})")
    gu.record_margin("dp3_bf16", loss_over_bar=max(a / b for a, b in loss_rows), worst_grad_over_bar=worst,
                     worst_bn_over_bar=bworst, autocast_chunked=[str(s) for s in fx["autocast_chunked"]])


def test_dp_bf16_checkpointed_decoder_bit_identical(tmp_path):
    """Config 5's mode (BASELINE configs[4]: bf16, data parallel, decoder activation
    checkpointing) at a small shape: the two-rank bf16 step with checkpoint_decoder=True leaves
    the same losses, mean gradient, Adam-step parameters and BatchNorm buffers, bit for bit, as
    the two-rank bf16 step without it (the recompute reuses the forward's BatchNorm
    coefficients; every reduction sums in a fixed order)."""
    plain = _run(tmp_path, 2, 0.0, "32,32,32", precision="bf16", ckpt=False, tag="plain")
    ck = _run(tmp_path, 2, 0.0, "32,32,32", precision="bf16", ckpt=True, tag="ckpt")
    assert plain["losses"] == ck["losses"]
    for key in ("grad", "params", "bn"):
        assert torch.equal(plain[key], ck[key]), key
    assert torch.isfinite(plain["grad"]).all()


def test_dp_trainer_train_loop_two_ranks(tmp_path):
    """Trainer.train() end to end on two ranks: the ranks agree on the averaged
    losses (so ReduceLROnPlateau and early stopping take the same decisions), on the final
    parameters and BatchNorm buffers, and only rank 0 writes checkpoints."""
    from pcms_amd.data import DEFAULT_MODALITIES, write_nifti
    rng = np.random.default_rng(0)
    data = tmp_path / "data"
    for i in range(4):
        for m in DEFAULT_MODALITIES:
            d = data / "BPH-PCA" / "BPH" / m
            d.mkdir(parents=True, exist_ok=True)
            write_nifti(str(d / f"c{i}.nii"), (rng.random((16, 16, 16)) * 10).astype(np.float32))
        ld = data / "BPH-PCA" / "ROI(BPH+PCA)" / "BPH"
        ld.mkdir(parents=True, exist_ok=True)
        lab = np.zeros((16, 16, 16), np.uint8)
        lab[4:10, 5:11, 3:9] = 1
        write_nifti(str(ld / f"c{i}.nii"), lab)
    save = tmp_path / "ckpt"
    out = str(tmp_path / "train.pt")
    env = dict(os.environ, MODE="train", DATA=str(data), SAVE=str(save))
    port = str(_port())
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "tools", "dp_worker.py"), str(r), "2", port, out],
                              env=env) for r in range(2)]
    assert [p.wait(timeout=240) for p in procs] == [0, 0]
    ranks = torch.load(out, weights_only=True)["ranks"]
    assert ranks[0] == ranks[1]
    assert np.isfinite(ranks[0]["best"])
    assert (save / "latest_checkpoint.pth").exists()


def test_rccl_backend_gradsync():
    """The "nccl" (RCCL) backend that bench.py / Trainer use under data parallelism, at the
    world size one GPU allows (1): group init through torch.distributed.run on 127.0.0.1, the
    bucketed GradSync all-reduce and the BatchNorm broadcast on the device."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr=127.0.0.1", f"--master-port={_port()}",
                        os.path.join(HERE, "tools", "rccl_worker.py")], env=env, capture_output=True, text=True,
                       timeout=180)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "rccl ok: world 1" in r.stdout
