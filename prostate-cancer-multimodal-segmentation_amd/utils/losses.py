"""Drop-in ``DiceLoss`` / ``BCEDiceLoss`` (utils/losses.py of the reference) on HIP kernels.

DiceLoss(smooth=1.0):   1 - (2 sum(p t) + s) / (sum p + sum t + s),  p = sigmoid(pred),
                        sums over the WHOLE batch (view(-1), utils/losses.py:72-92).
BCEDiceLoss(0.5, 0.5):  bce_weight * mean BCEWithLogits + dice_weight * Dice (:124-152).

Forward: one pass producing fp32 block partials of (sum p t, sum p, sum t, sum bce),
combined in fp64 on device; backward: one elementwise pass for dL/dpred.  No host sync.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import _lib
from .._lib import call, query


class _LossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, smooth, wb, wd):
        if pred.device.type != "cuda":
            raise RuntimeError("pcms_amd losses run on a ROCm device only (no CPU path)")
        x = pred.detach().contiguous().float()
        t = target.detach().contiguous().to(device=x.device, dtype=torch.float32)
        M = x.numel()
        rows = query("pcms_loss_rows", M)
        part = torch.empty(rows * 4, dtype=torch.float32, device=x.device)
        sums = torch.empty(4, dtype=torch.float64, device=x.device)
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        call("pcms_loss_fwd", x, t, M, float(smooth), float(wb), float(wd), part, sums, loss)
        ctx.save_for_backward(x, t, sums)
        ctx.cfg = (float(smooth), float(wb), float(wd))
        ctx.shape = pred.shape
        return loss

    @staticmethod
    def backward(ctx, gout):
        x, t, sums = ctx.saved_tensors
        smooth, wb, wd = ctx.cfg
        dx = torch.empty_like(x)
        g = gout.detach().contiguous().float()
        call("pcms_loss_bwd", x, t, x.numel(), sums, smooth, wb, wd, g, dx)
        return dx.view(ctx.shape), None, None, None, None


def _check(pred, target):
    if pred.shape != target.shape:
        raise ValueError(f"预测值和目标值的形状不匹配: pred.shape={pred.shape}, target.shape={target.shape}")


class DiceLoss(nn.Module):
    """Soft Dice loss on sigmoid(pred), global over the batch (utils/losses.py:16-92)."""

    def __init__(self, smooth: float = 1.0):
        super().__init__()
        self.smooth = smooth

    def forward(self, pred, target):
        _check(pred, target)
        return _LossFunction.apply(pred, target, self.smooth, 0.0, 1.0)


class BCEDiceLoss(nn.Module):
    """bce_weight * BCEWithLogits(mean) + dice_weight * Dice (utils/losses.py:95-152)."""

    def __init__(self, bce_weight: float = 0.5, dice_weight: float = 0.5):
        super().__init__()
        self.bce_weight = bce_weight
        self.dice_weight = dice_weight
        self.bce_loss = nn.BCEWithLogitsLoss()  # attribute parity; the fused kernel computes it
        self.dice_loss = DiceLoss()

    def forward(self, pred, target):
        _check(pred, target)
        return _LossFunction.apply(pred, target, self.dice_loss.smooth, self.bce_weight, self.dice_weight)
