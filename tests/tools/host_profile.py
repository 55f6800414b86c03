"""Host-side (Python) cost of one training step (test tooling): cProfile over steps whose GPU
work is already queued behind a long kernel, so host time is not hidden by GPU waits."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import pcms_amd  # noqa
    from pcms_amd.synthetic import make_batch
    from pcms_amd.utils.trainer import Trainer
    torch.manual_seed(0)
    tr = Trainer({"device": "cuda", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1, "loss": "bce_dice"})
    b = make_batch(2, (128, 128, 64), seed=1)
    batch = {"image": b["image"].cuda(), "label": b["label"].cuda()}
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        tr.step_async(batch)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / 5:.2f} ms/step, wall {1e3 * (t2 - t0) / 5:.2f} ms/step", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        tr.step_async(batch)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
