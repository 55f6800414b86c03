"""``GradScaler`` for the mixed-precision step variant of the reference
(train_bph_optimized.py:248 ``GradScaler('cuda')``, :269 ``autocast('cuda')``, :296-298
``scaler.scale(loss).backward(); scaler.step(optimizer); scaler.update()``).

The MI355X engine's reduced-precision path is bf16 storage with fp32 accumulation (the
``precision="bf16"`` build), not fp16: ``autocast`` has no role, the engine already runs
its convolutions in bf16.  The scaler keeps torch.amp.GradScaler's dynamic loss scaling
semantics: the loss is multiplied by ``scale`` before backward; ``step`` unscales the flat
gradient (folded into the fused norm pass and the Adam kernel, no extra pass), skips the
optimizer step when any gradient is inf/NaN, and ``update`` backs the scale off by 0.5 after
a skipped step or grows it by 2 after ``growth_interval`` clean ones.
"""
from __future__ import annotations

import math

import torch

from ._lib import call, query


class GradScaler:
    def __init__(self, device: str = "cuda", init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000, enabled: bool = True):
        self._scale = float(init_scale)
        self.growth_factor = float(growth_factor)
        self.backoff_factor = float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self.enabled = bool(enabled)
        self._growth_tracker = 0
        self._found_inf = None
        self._unscaled = False
        self._ws = self._norm = self._mul = None

    def get_scale(self) -> float:
        return self._scale if self.enabled else 1.0

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        return loss * self._scale if self.enabled else loss

    def _buffers(self, dev):
        if self._ws is None or self._ws.device != dev:
            self._ws = torch.empty(query("pcms_grad_clip_ws_doubles"), dtype=torch.float64, device=dev)
            self._norm = torch.empty(1, device=dev)
            self._mul = torch.empty(1, device=dev)
        return self._ws, self._norm, self._mul

    def unscale_(self, optimizer):
        """torch.amp.GradScaler.unscale_: divide the gradients by the scale (and apply the
        optimizer's pending data-parallel ``grad_scale``) IN PLACE, so ``param.grad`` holds
        the unscaled values afterwards and a following ``clip_grad_norm_`` measures and clips
        them (torch's documented unscale_ -> clip -> step sequence).  The norm of the unscaled
        gradient, taken in the same pass, tells ``step`` whether any element is inf/NaN."""
        self._unscale(optimizer, 0.0, in_place=True)

    def _unscale(self, optimizer, max_norm: float = 0.0, in_place: bool = False):
        """``in_place=False`` (Trainer's own step, and ``step`` without a prior unscale_):
        1/scale, the data-parallel grad_scale and a clip to ``max_norm`` (> 0) are folded into
        the optimizer's device-side gradient multiplier -- one norm pass, no scale pass; the
        Adam kernel writes the unscaled (clipped) gradient back into ``param.grad``."""
        if not self.enabled or self._unscaled:
            return
        eng = optimizer.model.engine()
        ws, norm, mul = self._buffers(eng.flat_g.device)
        gscale = float(optimizer.grad_scale) / self._scale
        call("pcms_grad_clip", eng.flat_g, eng.flat_g.numel(), gscale, float(max_norm), 1 if in_place else 0, ws,
             norm, mul)
        optimizer.grad_mul = None if in_place else mul
        optimizer.grad_scale = 1.0
        self._unscaled = True

    def step(self, optimizer, *args, **kwargs):
        if not self.enabled:
            return optimizer.step(*args, **kwargs)
        if all(p.grad is None for p in optimizer.model.parameters()):
            # no backward since zero_grad(set_to_none=True): flat_g holds a previous step's
            # values; torch's GradScaler raises here as well
            raise AssertionError("No inf checks were recorded for this optimizer.")
        self._unscale(optimizer)
        self._found_inf = not math.isfinite(float(self._norm))  # host sync, as torch's scaler
        if self._found_inf:
            optimizer.grad_mul = None
            optimizer.grad_scale = 1.0
            return None
        return optimizer.step(*args, **kwargs)

    def update(self, new_scale=None):
        if not self.enabled:
            return
        if new_scale is not None:
            self._scale = float(new_scale)
        elif self._found_inf:
            self._scale *= self.backoff_factor
            self._growth_tracker = 0
        elif self._found_inf is not None:
            self._growth_tracker += 1
            if self._growth_tracker == self.growth_interval:
                self._scale *= self.growth_factor
                self._growth_tracker = 0
        self._found_inf = None
        self._unscaled = False

    def state_dict(self):
        return {"scale": self._scale, "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": self._growth_tracker}

    def load_state_dict(self, sd):
        self._scale = float(sd["scale"])
        self.growth_factor = float(sd["growth_factor"])
        self.backoff_factor = float(sd["backoff_factor"])
        self.growth_interval = int(sd["growth_interval"])
        self._growth_tracker = int(sd["_growth_tracker"])


def clip_grad_norm_(model, max_norm: float, optimizer=None) -> torch.Tensor:
    """``torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm)`` (train_bph.py:166,
    train_bph_cv.py:311) on the engine's flat gradient: one fused fp64-partial norm pass and,
    when the gradient is clipped, one in-place scale pass.  ``optimizer``: a FlatAdam whose
    pending data-parallel ``grad_scale`` is applied first (the mean gradient is clipped).
    Returns the total norm (device tensor)."""
    eng = model.engine()
    dev = eng.flat_g.device
    ws = torch.empty(query("pcms_grad_clip_ws_doubles"), dtype=torch.float64, device=dev)
    norm = torch.empty(1, device=dev)
    mul = torch.empty(1, device=dev)
    gscale = 1.0
    if optimizer is not None:
        gscale, optimizer.grad_scale = float(optimizer.grad_scale), 1.0
    call("pcms_grad_clip", eng.flat_g, eng.flat_g.numel(), gscale, float(max_norm), 1, ws, norm, mul)
    return norm[0]
