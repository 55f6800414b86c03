"""pcms_amd — MI355X-native (gfx950) engine for the 5-channel prostate-MRI 3D U-Net of
qwertyhgb/Prostate-Cancer-Multimodal-Segmentation.

Drop-in surface (reference module paths mirrored):
  pcms_amd.models.unet3d  -> UNet3D, DoubleConv3D, Down3D, Up3D
  pcms_amd.utils.losses   -> DiceLoss, BCEDiceLoss
  pcms_amd.utils.trainer  -> BaseTrainer, Trainer (with step())
The compute runs in libpcms_hip.so (include/pcms_hip.h); importing this package loads it
and fails loudly if it is missing.
"""
from . import _lib

_lib.load()

from .models.unet3d import UNet3D, DoubleConv3D, Down3D, Up3D  # noqa: E402
from .utils.losses import DiceLoss, BCEDiceLoss  # noqa: E402
from .optim import FlatAdam  # noqa: E402
from .utils.trainer import BaseTrainer, Trainer  # noqa: E402

__all__ = ["UNet3D", "DoubleConv3D", "Down3D", "Up3D", "DiceLoss", "BCEDiceLoss", "FlatAdam",
           "BaseTrainer", "Trainer"]
