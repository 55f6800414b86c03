"""One rank of the RCCL check (tests/test_dp_gpu.py::test_rccl_backend_gradsync): joins a
"nccl" (= RCCL on ROCm) group at the world size the launcher set, runs the engine's
bucketed gradient all-reduce (pcms_amd.dp.GradSync) and the BatchNorm-buffer broadcast
through it on this rank's GPU, and checks the sums.  Env: WORLD_SIZE / RANK / LOCAL_RANK /
MASTER_* (torch.distributed.run)."""
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    world, rank = dist.get_world_size(), dist.get_rank()
    assert world == int(os.environ["WORLD_SIZE"]), (world, os.environ["WORLD_SIZE"])
    assert dist.get_backend() == "nccl"
    from pcms_amd.dp import GradSync
    n = 3 * (1 << 20) + 12345
    g = torch.arange(n, device=dev, dtype=torch.float32) * 1e-3 + rank
    sync = GradSync(g, bucket_elems=1 << 20)
    # the backward reports module ranges from the end of the buffer downwards
    edges = [n, n - 700000, n - 1900000, 1 << 19, 0]
    for hi, lo in zip(edges[:-1], edges[1:]):
        sync.ready(lo, hi)
    scale = sync.finish()
    torch.cuda.synchronize()
    assert scale == 1.0 / world
    assert len(sync.launched) >= 2, sync.launched
    want = torch.arange(n, device=dev, dtype=torch.float32) * 1e-3 * world + world * (world - 1) / 2
    assert torch.allclose(g, want, rtol=1e-6, atol=1e-4), float((g - want).abs().max())
    bn = torch.full((11794,), float(rank + 1), device=dev)
    sync.broadcast_buffers(bn)
    torch.cuda.synchronize()
    assert torch.all(bn == 1.0)
    dist.barrier()
    if rank == 0:
        print(f"rccl ok: world {world}, buckets {sync.launched}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
