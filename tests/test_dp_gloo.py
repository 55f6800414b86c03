"""Data-parallel step logic on CPU: world size 2 over gloo.

The product's DP layer (``pcms_amd.dp.GradSync``: rank-0 BatchNorm-buffer broadcast,
bucketed all-reduce of the flat gradient driven by the backward's module-completion
order, 1/world scale for Adam) runs here on CPU tensors with gradients produced by the
oracle (tests may call the oracle; the GPU engine cannot run in this container).  The
result of two DP steps on two ranks must equal ``oracle.dp_step_simulated``, the CPU
restatement of DistributedDataParallel(broadcast_buffers=True) around the reference
step (utils/trainer.py:183-192).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SPATIAL = (16, 16, 16)
STEPS = 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bn_keys(sd):
    return [k for k in sd if k.endswith(("running_mean", "running_var"))]


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(2)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import pcms_amd  # noqa: F401
        from oracle import unet3d_cpu as ref
        from pcms_amd.dp import BACKWARD_ORDER, GradSync, module_grad_ranges
        from pcms_amd.synthetic import make_batch, step_seed

        torch.manual_seed(0)
        sd = ref.init_params(5, 1)
        keys = ref.param_keys(sd)
        ranges = module_grad_ranges((k, sd[k]) for k in keys)
        total = sum(sd[k].numel() for k in keys)
        flat_g = torch.zeros(total)
        bn_keys = _bn_keys(sd)
        flat_bn = torch.cat([sd[k].reshape(-1) for k in bn_keys])
        sync = GradSync(flat_g, bucket_elems=1 << 20)
        for k in keys:
            sd[k].requires_grad_(True)
        opt = torch.optim.Adam([sd[k] for k in keys], lr=1e-4, weight_decay=1e-5)
        for s in range(STEPS):
            # rank 0's running buffers everywhere (DDP broadcast_buffers)
            flat_bn.copy_(torch.cat([sd[k].reshape(-1) for k in bn_keys]))
            sync.broadcast_buffers(flat_bn)
            off = 0
            with torch.no_grad():
                for k in bn_keys:
                    n = sd[k].numel()
                    sd[k].copy_(flat_bn[off:off + n].view_as(sd[k]))
                    off += n
            b = make_batch(2, SPATIAL, seed=step_seed(rank, s), label="bernoulli")
            opt.zero_grad()
            loss = ref.bce_dice_loss(ref.forward(sd, b["image"], training=True), b["label"])
            loss.backward()
            off = 0
            for k in keys:
                n = sd[k].numel()
                flat_g[off:off + n].copy_(sd[k].grad.reshape(-1))
                off += n
            for name in BACKWARD_ORDER:   # the engine's completion order
                sync.ready(*ranges[name])
            scale = sync.finish()
            assert scale == 1.0 / world
            assert len(sync.launched) >= 3, sync.launched   # bucketed, not one message
            off = 0
            for k in keys:
                n = sd[k].numel()
                sd[k].grad = flat_g[off:off + n].view_as(sd[k]) * scale
                off += n
            opt.step()
        # every rank holds the same parameters
        pv = torch.cat([sd[k].detach().reshape(-1) for k in keys])
        p0 = pv.clone()
        dist.broadcast(p0, src=0)
        assert torch.equal(pv, p0), "ranks diverged"
        if rank == 0:
            torch.manual_seed(0)
            sim = ref.init_params(5, 1)
            sopt = None
            for s in range(STEPS):
                shards = []
                for r in range(world):
                    bb = make_batch(2, SPATIAL, seed=step_seed(r, s), label="bernoulli")
                    shards.append((bb["image"], bb["label"]))
                _, sopt = ref.dp_step_simulated(sim, shards, lr=1e-4, loss="bce_dice", opt=sopt)
            worst = max(float((sd[k].detach() - sim[k].detach()).abs().max()) for k in keys)
            assert worst <= 1e-7, f"DP params differ from the DDP simulation by {worst}"
            # BN buffers: ours are rank 0's after its last forward = the simulation's
            for k in bn_keys:
                assert torch.equal(sd[k], sim[k]), k
        q.put((rank, "ok"))
    except BaseException as e:  # report to the parent
        q.put((rank, f"{type(e).__name__}: {e}"))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_dp_two_ranks_gloo_matches_ddp_simulation():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, msg = q.get(timeout=600)
            res[r] = msg
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert res == {0: "ok", 1: "ok"}, res


def test_backward_order_tiles_the_flat_buffer():
    """The engine reports module gradients in BACKWARD_ORDER; the ranges must tile the
    flat buffer from its end down to 0 (what GradSync.ready requires)."""
    import pcms_amd  # noqa: F401
    from oracle import unet3d_cpu as ref
    from pcms_amd.dp import BACKWARD_ORDER, module_grad_ranges

    sd = ref.init_params(5, 1)
    keys = ref.param_keys(sd)
    ranges = module_grad_ranges((k, sd[k]) for k in keys)
    assert set(ranges) == set(BACKWARD_ORDER)
    hi = sum(sd[k].numel() for k in keys)
    for name in BACKWARD_ORDER:
        lo, h = ranges[name]
        assert h == hi, name
        hi = lo
    assert hi == 0


def test_gradsync_rejects_out_of_order_ranges():
    import pcms_amd  # noqa: F401
    from pcms_amd.dp import GradSync
    port = _port()
    store = dist.TCPStore("127.0.0.1", port, 1, True)
    dist.init_process_group("gloo", store=store, rank=0, world_size=1)
    try:
        g = torch.arange(10, dtype=torch.float32)
        s = GradSync(g, bucket_elems=4)
        s.ready(6, 10)
        with pytest.raises(RuntimeError):
            s.ready(0, 5)   # gap: [5, 6) never reported
        s.ready(2, 6)
        assert s.finish() == 1.0
        assert s.launched == [(6, 10), (2, 6), (0, 2)], s.launched
        assert torch.equal(g, torch.arange(10, dtype=torch.float32))   # world 1: sum = identity
    finally:
        dist.destroy_process_group()
