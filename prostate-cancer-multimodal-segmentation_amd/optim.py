"""Flat-buffer Adam: ``torch.optim.Adam(params, lr, weight_decay=wd)`` semantics
(utils/trainer.py:113-117 — coupled L2: g += wd * p, bias-corrected moments, eps outside
the sqrt) applied to the engine's single fp32 master / grad buffers in ONE kernel launch.

``state_dict()`` uses torch.optim.Adam's format (per-parameter ``step``, ``exp_avg``,
``exp_avg_sq``), so reference checkpoints' ``optimizer_state_dict`` round-trips.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ._lib import call


class FlatAdam(torch.optim.Optimizer):
    def __init__(self, model: nn.Module, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        if not hasattr(model, "engine"):
            raise TypeError("FlatAdam needs a pcms_amd UNet3D (it updates the engine's flat buffers)")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(list(model.parameters()), defaults)
        self.model = model
        self.step_count = 0
        # gradient multipliers applied by the Adam kernel (one step): grad_scale (host float:
        # the data-parallel 1/world) and grad_mul (device fp32 scalar from pcms_grad_clip: the
        # clip coefficient / AMP unscale), both folded into the single Adam pass
        self.grad_scale = 1.0
        self.grad_mul = None
        self.fused_packs = True  # Adam writes the conv / ConvT packs (engine.adam_plan; both builds)
        self._m = None
        self._v = None

    def _moments(self, eng):
        n = eng.flat_p.numel()
        if self._m is None or self._m.numel() != n or self._m.device != eng.flat_p.device:
            self._m = torch.zeros(n, dtype=torch.float32, device=eng.flat_p.device)
            self._v = torch.zeros(n, dtype=torch.float32, device=eng.flat_p.device)
        return self._m, self._v

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if len(self.param_groups) != 1:
            raise ValueError("FlatAdam supports a single parameter group")
        g = self.param_groups[0]
        if all(p.grad is None for p in self.param_groups[0]["params"]):
            return loss  # torch.optim.Adam skips parameters without a gradient
        eng = self.model.engine(full_sync=False)
        m, v = self._moments(eng)
        self.step_count += 1
        b1, b2 = g["betas"]
        bc1 = 1.0 - b1 ** self.step_count
        bc2 = 1.0 - b2 ** self.step_count
        coef = (g["lr"] / bc1, b1, b2, g["eps"], g["weight_decay"], math.sqrt(bc2), float(self.grad_scale))
        plan = eng.adam_plan() if self.fused_packs else None
        if plan is not None:
            # bf16 build: the conv / ConvT weight packs come out of the Adam pass itself
            P = (eng.flat_p, eng.flat_g, m, v)
            sfx = "_x6" if plan["x6"] else ""  # fp32 build: the bf16x6 packs
            call("pcms_adam_pack_conv3" + sfx, *P, plan["conv"], plan["nconv"], plan["conv_tiles"], *coef,
                 self.grad_mul)
            call("pcms_adam_pack_convt" + sfx, *P, plan["convt"], plan["nconvt"], plan["convt_tiles"], *coef,
                 self.grad_mul)
            call("pcms_adam_ranges", *P, plan["ranges"], plan["nranges"], plan["max_len"], *coef, self.grad_mul)
        else:
            call("pcms_adam", eng.flat_p, eng.flat_g, m, v, eng.flat_p.numel(), *coef, self.grad_mul)
        # one-shot multipliers of this step's gradient (the kernel wrote the scaled gradient
        # back into param.grad)
        self.grad_scale = 1.0
        self.grad_mul = None
        eng.mark_dirty(packs_fresh=plan is not None and plan["complete"])
        return loss

    def zero_grad(self, set_to_none: bool = True):
        """torch semantics: ``set_to_none`` (the default) leaves every ``param.grad`` None --
        the next backward then writes the flat gradient instead of accumulating into it, so
        no zero fill runs; ``set_to_none=False`` zeroes the flat gradient in place."""
        eng = self.model._engine
        if eng is not None and not set_to_none:
            eng.flat_g.zero_()
            eng.sync_params(full=False)
        else:
            for p in self.model.parameters():
                p.grad = None

    # ---- torch.optim.Adam-compatible (de)serialisation ----
    def state_dict(self):
        g = dict(self.param_groups[0])
        params = g.pop("params")
        g["params"] = list(range(len(params)))
        state = {}
        if self._m is not None:
            off = 0
            for i, p in enumerate(params):
                n = p.numel()
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": self._m[off:off + n].view_as(p).clone(),
                            "exp_avg_sq": self._v[off:off + n].view_as(p).clone()}
                off += n
        return {"state": state, "param_groups": [g]}

    def load_state_dict(self, state_dict):
        groups = state_dict["param_groups"]
        if len(groups) != 1:
            raise ValueError("FlatAdam expects one param group")
        for k, val in groups[0].items():
            if k != "params":
                self.param_groups[0][k] = val
        st = state_dict["state"]
        if not st:
            return
        eng = self.model.engine()
        m, v = self._moments(eng)
        off = 0
        with torch.no_grad():
            for i, p in enumerate(self.param_groups[0]["params"]):
                n = p.numel()
                s = st[i] if i in st else st[str(i)]
                m[off:off + n].copy_(s["exp_avg"].reshape(-1))
                v[off:off + n].copy_(s["exp_avg_sq"].reshape(-1))
                off += n
            step = st[0]["step"] if 0 in st else st["0"]["step"]
        self.step_count = int(float(step))
