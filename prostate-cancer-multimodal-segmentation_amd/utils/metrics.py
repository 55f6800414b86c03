"""Validation metrics and the evaluation loop (reference
script/validate_model.py:24-95 metrics, :188-274 per-case evaluation).

Binary masks come from ``UNet3D.inference`` (HIP eval forward: BatchNorm from running stats,
``logit > 0`` for threshold 0.5); the two overlap scores are small reductions over those
masks, done where the masks live (device tensors, no host round trip per voxel).
"""
from __future__ import annotations

from typing import Dict, Iterable, List

import torch


def calculate_dice_score(pred: torch.Tensor, target: torch.Tensor) -> float:
    """2|X∩Y| / (|X| + |Y| + 1e-8) over all voxels (validate_model.py:24-50)."""
    p, t = pred.reshape(-1).float(), target.reshape(-1).float()
    inter = (p * t).sum()
    return float((2.0 * inter) / (p.sum() + t.sum() + 1e-8))


def calculate_iou(pred: torch.Tensor, target: torch.Tensor) -> float:
    """|X∩Y| / (|X∪Y| + 1e-8) (validate_model.py:53-80)."""
    p, t = pred.reshape(-1).float(), target.reshape(-1).float()
    inter = (p * t).sum()
    union = p.sum() + t.sum() - inter
    return float(inter / (union + 1e-8))


@torch.no_grad()
def evaluate(model, loader: Iterable, threshold: float = 0.5, device=None) -> Dict:
    """Per-case Dice / IoU of ``model.inference`` masks against binarised labels, and their
    means (the ModelValidator loop, validate_model.py:226-274, one case per batch item)."""
    device = device or next(model.parameters()).device
    model.eval()
    cases: List[Dict] = []
    for batch in loader:
        x = batch["image"].to(device, non_blocking=True)
        y = batch["label"].to(device, non_blocking=True)
        mask = model.inference(x, threshold=threshold)
        ids = batch.get("case_id", [str(len(cases) + i) for i in range(x.shape[0])])
        for i in range(x.shape[0]):
            cases.append({"case_id": ids[i], "dice": calculate_dice_score(mask[i], y[i]),
                          "iou": calculate_iou(mask[i], y[i])})
    n = max(len(cases), 1)
    return {"cases": cases, "mean_dice": sum(c["dice"] for c in cases) / n,
            "mean_iou": sum(c["iou"] for c in cases) / n}
