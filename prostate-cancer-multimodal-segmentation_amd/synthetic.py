"""Synthetic batches for the bench and the parity tests.

* image  ~ U[0, 1) float32, NCDHW (N, 5, D, H, W) — the min-max range the reference
  predictor feeds the model (script/predict.py:70-75);
* label  float32 {0, 1}, NCDHW (N, 1, D, H, W): a centred ellipsoid with semi-axes
  (0.30 D, 0.25 H, 0.25 W), each jittered by ±10 % (≈8 % foreground), or a
  Bernoulli(0.5) mask (gradient-rich parity variant);
* per-step seed ``1234 + 1000 * rank + step``;
* ``zero_fill``: per sample, k ∈ {1, 2} random modalities set to all-zero channels,
  the missing-modality semantics of script/data_loader.py:320-322.

Returns the batch dict the reference loader yields (script/data_loader.py:415-419).
"""
from __future__ import annotations

import torch


def step_seed(rank: int, step: int) -> int:
    return 1234 + 1000 * rank + step


def make_batch(n: int, spatial=(128, 128, 64), n_modalities: int = 5, seed: int = 1234,
               label: str = "ellipsoid", zero_fill: bool = False) -> dict:
    g = torch.Generator().manual_seed(seed)
    d, h, w = spatial
    image = torch.rand((n, n_modalities, d, h, w), generator=g, dtype=torch.float32)
    if label == "bernoulli":
        lab = (torch.rand((n, 1, d, h, w), generator=g) < 0.5).float()
    else:
        lab = torch.zeros((n, 1, d, h, w), dtype=torch.float32)
        zz = torch.arange(d, dtype=torch.float32).view(d, 1, 1) - (d - 1) / 2
        yy = torch.arange(h, dtype=torch.float32).view(1, h, 1) - (h - 1) / 2
        xx = torch.arange(w, dtype=torch.float32).view(1, 1, w) - (w - 1) / 2
        for i in range(n):
            j = 1.0 + 0.2 * (torch.rand(3, generator=g) - 0.5)
            a = (0.30 * d * j[0], 0.25 * h * j[1], 0.25 * w * j[2])
            r = (zz / a[0]) ** 2 + (yy / a[1]) ** 2 + (xx / a[2]) ** 2
            lab[i, 0] = (r <= 1.0).float()
    cases = [f"synthetic_{seed}_{i}" for i in range(n)]
    if zero_fill:
        for i in range(n):
            k = int(torch.randint(1, 3, (1,), generator=g))
            drop = torch.randperm(n_modalities, generator=g)[:k]
            image[i, drop] = 0.0
    return {"image": image, "label": lab, "case_id": cases}
