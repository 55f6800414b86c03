"""Single-case prediction pipeline (reference script/predict.py), on the HIP engine.

* ``load_multimodal_images(case_dir, handle_missing)``: the five modality folders
  ['ADC', 'DWI', 'gaoqing-T2', 'T2 fs', 'T2 not fs'] (predict.py:25), the first ``.nii`` of
  each, per-modality min-max normalisation to [0, 1] (constant image -> zeros, :70-75),
  missing modalities by 'zero_fill' / 'skip' / 'duplicate' (:38-55), stacked (5, D, H, W)
  (:81).  NIfTI through pcms_amd.data's reader (SimpleITK is not a dependency).
* ``preprocess_image``: (1, 5, D, H, W) float32 tensor (:85-100).
* ``ModelPredictor(model_path, device)``: UNet3D(n_modalities=5, n_classes=1) with either
  checkpoint form (:121-145), ``predict`` -> (D, H, W) probabilities from ``UNet3D.predict``
  (sigmoid in the head kernel, :160-170), ``save_prediction`` -> uint8 ``> 0.5`` mask NIfTI
  with the reference image's voxel spacing when one is given (:172-196).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import numpy as np
import torch

from .data import read_nifti, read_nifti_header, write_nifti
from .models.unet3d import UNet3D, load_weights

MODALITIES = ["ADC", "DWI", "gaoqing-T2", "T2 fs", "T2 not fs"]


def load_multimodal_images(case_dir: str, handle_missing: str = "zero_fill") -> Tuple[np.ndarray, List[str]]:
    images, reference = [], None
    for modality in MODALITIES:
        mdir = os.path.join(case_dir, modality)
        if not os.path.exists(mdir):
            raise FileNotFoundError(f"modality directory missing: {mdir}")
        files = sorted(f for f in os.listdir(mdir) if f.endswith(".nii"))
        if not files:
            if handle_missing == "zero_fill":
                img = np.zeros_like(reference, dtype=np.float32) if reference is not None else \
                    np.zeros((64, 64, 64), dtype=np.float32)
            elif handle_missing == "duplicate" and reference is not None:
                img = reference.copy()
            else:
                raise FileNotFoundError(f"no .nii file in {mdir}")
        else:
            img = read_nifti(os.path.join(mdir, files[0]))
            if reference is None:
                reference = img
        img = img.astype(np.float32)
        lo, hi = float(img.min()), float(img.max())
        img = (img - lo) / (hi - lo) if hi - lo != 0 else np.zeros_like(img, dtype=np.float32)
        images.append(img.astype(np.float32))
    return np.stack(images, axis=0), list(MODALITIES)


def preprocess_image(image: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(image)).float().unsqueeze(0)


class ModelPredictor:
    def __init__(self, model_path: str, device: str = "cuda", precision: str = "bf16"):
        self.device = torch.device(device)
        self.model = UNet3D(n_modalities=5, n_classes=1, precision=precision).to(self.device)
        load_weights(self.model, model_path)
        self.model.eval()

    def predict(self, image_tensor: torch.Tensor) -> np.ndarray:
        with torch.no_grad():
            out = self.model.predict(image_tensor.to(self.device))
        return out.squeeze(0).squeeze(0).cpu().numpy()

    def save_prediction(self, prediction: np.ndarray, output_path: str,
                        reference_image_path: Optional[str] = None) -> None:
        spacing = (1.0, 1.0, 1.0)
        if reference_image_path and os.path.exists(reference_image_path):
            spacing = read_nifti_header(reference_image_path)["spacing"][:3]
        write_nifti(output_path, (prediction > 0.5).astype(np.uint8), spacing=spacing)
