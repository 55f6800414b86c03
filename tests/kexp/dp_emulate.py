"""Data-parallel step at W GPUs emulated on ONE GPU (test tooling): the bf16 training step with
the engine's per-layer gradient readiness driving dp.GradSync's bucket rule, each bucket's
all-reduce replaced by K RCCL-footprint workgroups (tests/kexp/cu_hog.hip rccl_like_kernel:
ncclDevKernel_Generic's 37.6 KB of LDS and ~248 VGPRs) spinning on a side stream for the ring
all-reduce time of that bucket at W ranks, 2 (W - 1) / W x bytes / busbw + lat.  What it
measures: the step time the backward loses to CUs held by the collective (every persistent or
one-round grid of the library straggles behind a held CU) plus the exposed tail -- not xGMI.

    make -C tests/kexp libcuhog.so && python tests/kexp/dp_emulate.py [--world 8] [--busbw 350] [--k 16]

Policies: none (W = 1), overlap (GradSync: buckets launched as the backward finishes each
layer), end (dp_overlap=False: one all-reduce of the whole gradient after the backward)."""
import argparse
import ctypes
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


class FakeSync:
    """dp.GradSync's launch rule with each all-reduce replaced by an RCCL-footprint hog."""

    def __init__(self, hog, n, k, world, busbw, lat_us, bucket, min_bucket, overlap, sink):
        from pcms_amd.dp import _due
        self._due = _due
        self.hog, self.n, self.k, self.w = hog, n, k, world
        self.busbw, self.lat, self.bucket, self.minb, self.overlap, self.sink = busbw, lat_us, bucket, min_bucket, overlap, sink
        self.side = torch.cuda.Stream()
        self.reset()

    def reset(self):
        self.lo = self.hi = None
        self.launched = []
        self.us = 0.0

    def _launch(self, lo, hi):
        us = 2 * (self.w - 1) / self.w * (hi - lo) * 4 / (self.busbw * 1e9) * 1e6 + self.lat
        self.side.wait_stream(torch.cuda.current_stream())
        self.hog.cu_hog_rccl(self.k, us, self.sink.data_ptr(), self.side.cuda_stream)
        self.launched.append((lo, hi))
        self.us += us

    def ready(self, lo, hi):
        if self.hi is None:
            self.hi = hi
        self.lo = lo
        if self.overlap and self._due(self.hi - self.lo, self.lo, self.bucket, self.minb):
            self._launch(self.lo, self.hi)
            self.lo = self.hi = None

    def finish(self):
        if self.overlap:
            if self.hi is not None and self.hi > self.lo:
                self._launch(0, self.hi)
        else:
            self._launch(0, self.n)
        torch.cuda.current_stream().wait_stream(self.side)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--busbw", type=float, default=350.0, help="RCCL all-reduce bus bandwidth, GB/s")
    ap.add_argument("--lat", type=float, default=25.0, help="per-collective latency, us")
    ap.add_argument("--k", type=int, default=16, help="RCCL channels (workgroups) per collective")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--policies", default="none,overlap,end")
    ap.add_argument("--buckets", default="16", help="bucket sizes to compare (Mi elements, comma list): the "
                    "overlap policy is run once per size")
    a = ap.parse_args()
    import pcms_amd  # noqa: F401
    from pcms_amd.synthetic import make_batch
    from pcms_amd.utils.trainer import Trainer
    hog = ctypes.CDLL(os.path.join(HERE, "libcuhog.so"))
    hog.cu_hog_rccl.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    torch.manual_seed(0)
    tr = Trainer({"device": "cuda", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1,
                  "loss": "bce_dice", "precision": "bf16"})
    eng = tr.model.engine()
    b = make_batch(2, (128, 128, 64), seed=1)
    x, y = b["image"].cuda(), b["label"].cuda()
    sink = torch.zeros(64, dtype=torch.int32, device="cuda")
    n = eng.flat_g.numel()
    syncs = {"end": FakeSync(hog, n, a.k, a.world, a.busbw, a.lat, 16 << 20, 1 << 20, False, sink)}
    pols = []
    for p in a.policies.split(","):
        if p == "overlap":
            for bm in a.buckets.split(","):
                name = f"overlap{bm}M"
                syncs[name] = FakeSync(hog, n, a.k, a.world, a.busbw, a.lat, int(float(bm) * (1 << 20)),
                                       min(1 << 20, int(float(bm) * (1 << 20))), True, sink)
                pols.append(name)
        else:
            pols.append(p)

    def step(pol):
        tr.optimizer.zero_grad()
        s = syncs.get(pol)
        if s is not None:
            s.reset()
            eng.grad_ready = s.ready
        loss = tr.criterion(tr.model(x), y)
        loss.backward()
        eng.grad_ready = None
        if s is not None:
            s.finish()
        tr.optimizer.step()

    res = {p: [] for p in pols}
    for r in range(a.rounds):
        for p in pols:
            for _ in range(2):
                step(p)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                step(p)
            e1.record()
            e1.synchronize()
            res[p].append(e0.elapsed_time(e1) / a.steps)
    base = statistics.median(res[pols[0]])
    for p in pols:
        m = statistics.median(res[p])
        extra = ""
        if p in syncs:
            s = syncs[p]
            extra = (f"  buckets {len(s.launched)} ({[round((hi - lo) * 4 / 2**20, 1) for lo, hi in s.launched]} MB), "
                     f"all-reduce {s.us / 1e3:.2f} ms emulated")
        print(f"W={a.world} busbw {a.busbw:.0f} GB/s K={a.k} {p:8s} {m:7.3f} ms/step ({m / base - 1:+.1%} vs {pols[0]})"
              f"  all {[round(v, 3) for v in res[p]]}{extra}", flush=True)


if __name__ == "__main__":
    main()
