"""Validation metrics and the evaluation loop (reference
script/validate_model.py:24-95 metrics, :188-274 per-case evaluation).

Binary masks come from ``UNet3D.inference`` (HIP eval forward: BatchNorm from running stats,
``sigmoid > threshold`` in the head kernel); the two overlap scores are small reductions over those
masks, done where the masks live (device tensors, no host round trip per voxel).
"""
from __future__ import annotations

import json
import os
from datetime import datetime
from typing import Dict, Iterable, List, Optional

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


class ModelValidator:
    """script/validate_model.py:98-274: load a checkpoint (either form), run the test loader
    through ``UNet3D.inference`` (HIP eval forward, sigmoid > 0.5 in the head kernel), per-case
    Dice / IoU, and write ``validation_results.json`` to ``config['save_dir']`` with the
    reference's keys (timestamp, avg_dice, avg_iou, case_count, case_results)."""

    def __init__(self, config: dict, model=None, test_loader: Optional[Iterable] = None):
        from ..models.unet3d import UNet3D, load_weights
        self.config = config
        self.device = torch.device(config.get("device", "cuda"))
        if model is None:
            model = UNet3D(n_modalities=5, n_classes=1, precision=config.get("precision", "bf16")).to(self.device)
            if config.get("model_path"):
                load_weights(model, config["model_path"])
        self.model = model
        self.model.eval()
        if test_loader is None and config.get("data_dir"):
            from ..data import get_dataloader
            test_loader = get_dataloader(config["data_dir"], batch_size=config.get("batch_size", 1), shuffle=False,
                                         missing_strategy=config.get("handle_missing_modalities", "zero_fill"),
                                         target_size=tuple(config.get("target_size", (128, 128, 128))),
                                         is_training=False, data_type=config.get("data_type", "BPH"))
        self.test_loader = test_loader

    def validate(self):
        r = evaluate(self.model, self.test_loader, threshold=0.5, device=self.device)
        results = {"timestamp": datetime.now().strftime("%Y-%m-%d %H:%M:%S"), "avg_dice": r["mean_dice"],
                   "avg_iou": r["mean_iou"], "case_count": len(r["cases"]), "case_results": r["cases"]}
        save_dir = self.config.get("save_dir")
        if save_dir:
            os.makedirs(save_dir, exist_ok=True)
            with open(os.path.join(save_dir, "validation_results.json"), "w", encoding="utf-8") as f:
                json.dump(results, f, ensure_ascii=False, indent=2)
        return r["mean_dice"], r["mean_iou"]
