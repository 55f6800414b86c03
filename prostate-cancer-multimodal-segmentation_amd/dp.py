"""Data parallelism for the U-Net step: one process per GPU, ``torch.distributed`` with
the "nccl" (= RCCL on ROCm) backend; gloo on CPU for the tests.

The reference has no multi-GPU code.  The semantics chosen are those of
``DistributedDataParallel(model, broadcast_buffers=True)`` around the reference step
(utils/trainer.py:183-192), restated for the tests by
``oracle.unet3d_cpu.dp_step_simulated``:

* rank 0's BatchNorm running buffers are broadcast before every forward (ONE broadcast of
  the engine's flat BN buffer);
* every rank runs forward / loss / backward on its own volumes (per-replica BN statistics
  and per-replica global Dice);
* the flat fp32 gradient is summed over ranks; the 1/world mean is folded into Adam.

The gradient all-reduce is bucketed and overlapped with the backward: the engine reports
each LAYER's gradient range (a conv's weight + bias, a BatchNorm's gamma + beta, the
ConvTranspose, the head) as soon as the kernel that writes it is enqueued -- descending flat
order, the head first and the stem last (``readiness_groups``) -- and a bucket is launched
asynchronously (``async_op=True``: the RCCL kernel is ordered after the producing kernels of
the compute stream, then runs beside the rest of the backward).  A bucket goes out once it
holds ``bucket_elems`` elements, or once it holds ``min_bucket_elems`` and at most as many
elements remain to come as it holds: near the end of the backward the buckets shrink with
the remaining gradient, so the one bucket nothing overlaps (what ``finish`` launches) is the
last layers' (the stem and down1: ~0.3 M elements at the UNet3D sizes, not the ~14 M of the
four encoder modules it was with per-module readiness).  ``finish()`` makes the compute stream wait for every bucket before Adam,
which applies the 1/world mean in its single pass over the gradient and writes the mean
back, so ``param.grad`` holds the DDP mean after ``optimizer.step()``.
Buckets are contiguous slices of the flat gradient, so every collective is one large
message: xGMI rings are per-link bound, so few large transfers beat many small ones.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

# top-level modules in the order the engine's backward finishes their gradients
BACKWARD_ORDER = ("outc", "up4", "up3", "up2", "up1", "down4", "down3", "down2", "down1", "inc")


def readiness_groups(named) -> List[Tuple[str, int, int]]:
    """The (layer, lo, hi) flat ranges in the order the engine's backward reports them: one
    group per layer (parameters sharing a module prefix, e.g. ``down2.maxpool_conv.1.conv.3``
    = that conv's weight and bias), in descending flat order -- outc, up4's second BatchNorm,
    its second conv, ..., up4's ConvTranspose, up3 ..., down4 ..., inc's first conv.  ``named``:
    (name, tensor) pairs in parameter order (``model.named_parameters()``)."""
    groups: List[List] = []
    off = 0
    for name, p in named:
        layer = name.rsplit(".", 1)[0]
        if groups and groups[-1][0] == layer:
            groups[-1][2] = off + p.numel()
        else:
            groups.append([layer, off, off + p.numel()])
        off += p.numel()
    return [(g[0], g[1], g[2]) for g in reversed(groups)]


def plan_buckets(ranges, total: int, bucket_elems: int, min_bucket_elems: int) -> List[Tuple[int, int]]:
    """The buckets GradSync launches for ready ranges reported in this order (descending,
    tiling [0, total)), ending with the remainder finish() launches: the launch rule in one
    place for the tests."""
    out, lo, hi = [], None, None
    for a, b in ranges:
        if hi is None:
            hi = b
        lo = a
        if _due(hi - lo, lo, bucket_elems, min_bucket_elems):
            out.append((lo, hi))
            lo = hi = None
    if hi is not None and hi > lo:
        out.append((lo, hi))
    return out


def _due(pending: int, remaining: int, bucket_elems: int, min_bucket_elems: int) -> bool:
    return pending >= bucket_elems or (pending >= min_bucket_elems and remaining <= pending)


def module_grad_ranges(model) -> Dict[str, Tuple[int, int]]:
    """Element range [lo, hi) of each top-level module's parameters in the flat buffer
    (``model.parameters()`` order = the engine's flat layout).  ``model``: a module, or
    an iterable of (name, tensor) pairs in parameter order."""
    named = model.named_parameters() if hasattr(model, "named_parameters") else model
    ranges: Dict[str, List[int]] = {}
    off = 0
    for name, p in named:
        top = name.split(".", 1)[0]
        r = ranges.setdefault(top, [off, off])
        if r[1] != off:
            raise ValueError(f"parameters of {top} are not contiguous in the flat buffer")
        off += p.numel()
        r[1] = off
    return {k: (v[0], v[1]) for k, v in ranges.items()}


class GradSync:
    """Bucketed, backward-overlapped all-reduce (sum) of a flat gradient buffer.

    ``ready(lo, hi)`` declares flat_g[lo:hi] final.  Ranges arrive in descending order
    and tile the buffer (hi == the previous range's lo), as the U-Net backward produces
    them (outc and up4 sit at the end of the buffer, inc at offset 0).  Pending ranges are
    launched once they reach ``bucket_elems`` (default 16 Mi elements = 64 MB fp32), or
    ``min_bucket_elems`` (default 1 Mi) when no more than that many elements remain below
    them; ``finish()`` launches the rest, waits, and returns the 1/world scale Adam applies.
    """

    def __init__(self, flat_g: torch.Tensor, group=None, bucket_elems: int = 16 << 20, overlap: bool = True,
                 min_bucket_elems: int = 1 << 20):
        self.flat_g = flat_g
        self.group = group
        self.world = dist.get_world_size(group)
        self.bucket_elems = int(bucket_elems)
        self.min_bucket_elems = int(min(min_bucket_elems, bucket_elems))
        self.overlap = overlap
        self._works: List = []
        self._lo: Optional[int] = None   # pending range [lo, hi)
        self._hi: Optional[int] = None
        self._next_hi = flat_g.numel()   # the next ready range must end here
        self.launched: List[Tuple[int, int]] = []   # buckets of the current step (tests / logs)
        # bench.py under world > 1: HIP events on the compute stream around finish()'s waits
        # (the all-reduce time the backward did not hide), one (start, end) pair per step
        self.exposed_events: Optional[List] = None

    def reset(self):
        """Drop the state of a step whose backward stopped part-way (an exception between
        the first ``ready`` and ``finish``): wait for the buckets already launched (their
        sums land in a gradient the next step zeroes anyway), forget the pending range."""
        for w in self._works:
            w.wait()
        self._works = []
        self._lo = self._hi = None
        self._next_hi = self.flat_g.numel()
        self.launched = []

    def broadcast_buffers(self, flat_bn: torch.Tensor):
        """DDP broadcast_buffers: every rank takes rank 0's BatchNorm running statistics."""
        dist.broadcast(flat_bn, src=0, group=self.group)

    def _fresh_step(self):
        if self._next_hi == self.flat_g.numel() and not self._works:
            self.launched = []

    def ready(self, lo: int, hi: int):
        if hi != self._next_hi or not 0 <= lo <= hi:
            raise RuntimeError(f"gradient range [{lo}, {hi}) out of order (expected one ending at {self._next_hi})")
        self._fresh_step()
        self._next_hi = lo
        if self._hi is None:
            self._hi = hi
        self._lo = lo
        if self.overlap and _due(self._hi - self._lo, self._lo, self.bucket_elems, self.min_bucket_elems):
            self._launch()

    def _launch(self):
        if self._hi is not None and self._hi > self._lo:
            lo, hi = self._lo, self._hi
            self._works.append(dist.all_reduce(self.flat_g[lo:hi], op=dist.ReduceOp.SUM, group=self.group,
                                               async_op=True))
            self.launched.append((lo, hi))
        self._lo = self._hi = None

    def finish(self) -> float:
        """Launch what is pending (a range the backward did not report is reduced too),
        make the caller wait for every bucket, reset for the next step."""
        self._fresh_step()
        if self._next_hi != 0:
            if self._hi is None:
                self._hi = self._next_hi
            self._lo = 0
            self._next_hi = 0
        self._launch()
        ev = None
        if self.exposed_events is not None and self.flat_g.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for w in self._works:
            w.wait()
        if ev is not None:
            ev[1].record()
            self.exposed_events.append(ev)
        self._works = []
        self._next_hi = self.flat_g.numel()
        return 1.0 / self.world
