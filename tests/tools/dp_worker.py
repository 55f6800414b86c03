"""One rank of the data-parallel GPU test (tests/test_dp_gpu.py): Trainer.step's distributed
path on cuda:0 over gloo (CUDA tensors), ranks sharing one GPU.  Argv: rank world port out."""
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

SPATIAL = (32, 32, 16)


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    import pcms_amd  # noqa: F401
    from pcms_amd.synthetic import make_batch, step_seed
    from pcms_amd.utils.trainer import Trainer
    torch.manual_seed(0)
    cfg = {"device": "cuda:0", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1, "loss": "bce_dice",
           "precision": "fp32", "dp_bucket_elems": 4 << 20, "max_grad_norm": float(os.environ.get("CLIP", "0")) or None}
    tr = Trainer(cfg)
    assert tr.distributed and tr.world_size == world
    losses = []
    for s in range(int(os.environ.get("STEPS", "1"))):
        b = make_batch(2, SPATIAL, seed=step_seed(rank, s), label="bernoulli")
        losses.append(tr.step(b))
    eng = tr.model.engine()
    torch.cuda.synchronize()
    assert len(tr._sync.launched) >= 3, tr._sync.launched   # bucketed, overlapped with the backward
    p0 = eng.flat_p.clone()
    dist.broadcast(p0, src=0)
    assert torch.equal(p0, eng.flat_p), "ranks diverged"
    allp = [None] * world
    dist.all_gather_object(allp, losses)
    if rank == 0:
        torch.save({"losses": allp, "grad": eng.flat_g.cpu(), "params": eng.flat_p.cpu(), "bn": eng.flat_bn.cpu(),
                    "norm": None if tr.last_grad_norm is None else float(tr.last_grad_norm)}, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
