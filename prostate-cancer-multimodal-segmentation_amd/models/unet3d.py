"""Drop-in ``UNet3D`` for models/unet3d.py of the reference, executed by HIP kernels.

Same constructor (``UNet3D(n_modalities=5, n_classes=2)``; ``in_channels`` /
``out_channels`` accepted as aliases), same attributes (``n_modalities``, ``n_classes``,
``init_features = 64``), same submodule names and ``state_dict`` keys / shapes (136 keys
for n_classes=1), same initialisation under the same RNG state (models/unet3d.py:227-245:
kaiming_normal(fan_out) for Conv3d, BN (1, 0), ConvTranspose3d left at its default), and
the same ``forward`` / ``predict`` / ``inference`` semantics (models/unet3d.py:247-344).

What differs is where it runs: ``forward`` executes the whole network on a ROCm device via
``pcms_amd.engine.UNetEngine`` (NDHWC bf16 by default, or fp32 with
``precision="fp32"``); there is no CPU path.  ``predict`` / ``inference`` get their
sigmoid / threshold from the output-head kernel.  The sub-modules ``DoubleConv3D``,
``Down3D`` and ``Up3D`` are callable on their own (forward, train or eval BatchNorm, through
``pcms_amd.blocks``); training runs through ``UNet3D.forward`` as a whole.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .. import blocks
from ..engine import UNetEngine


class DoubleConv3D(nn.Module):
    """conv3x3x3(p=1) -> BN -> ReLU, twice (models/unet3d.py:5-55)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Sequential(
            nn.Conv3d(in_channels, out_channels, kernel_size=3, padding=1),
            nn.BatchNorm3d(out_channels),
            nn.ReLU(inplace=True),
            nn.Conv3d(out_channels, out_channels, kernel_size=3, padding=1),
            nn.BatchNorm3d(out_channels),
            nn.ReLU(inplace=True),
        )

    def forward(self, x):
        return blocks.double_conv_forward(self, x)


class Down3D(nn.Module):
    """MaxPool3d(2) -> DoubleConv3D (models/unet3d.py:57-96)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool3d(2), DoubleConv3D(in_channels, out_channels))

    def forward(self, x):
        return blocks.down_forward(self, x)


class Up3D(nn.Module):
    """ConvTranspose3d(k2, s2) -> pad -> cat[skip, up] -> DoubleConv3D (models/unet3d.py:98-158)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.up = nn.ConvTranspose3d(in_channels, in_channels // 2, kernel_size=2, stride=2)
        self.conv = DoubleConv3D(in_channels, out_channels)

    def forward(self, x1, x2):
        return blocks.up_forward(self, x1, x2)


class _UNetFunction(torch.autograd.Function):
    """Autograd node of one training forward; backward runs the HIP backward schedule and
    writes parameter gradients straight into the flat gradient buffer (``param.grad``)."""

    @staticmethod
    def forward(ctx, x, engine, *params):
        logits = engine.forward(x, training=True)
        ctx.engine = engine
        ctx.epoch = engine.epoch
        ctx.nparams = len(params)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        if ctx.engine.epoch != ctx.epoch:
            raise RuntimeError("UNet3D: another forward ran before this graph's backward; "
                               "the engine keeps only the latest forward's activations")
        ctx.engine.backward(dlogits)
        return (None, None) + (None,) * ctx.nparams


class UNet3D(nn.Module):
    """3D U-Net, 4 down / 4 up levels, widths 64 -> 1024 (models/unet3d.py:160-344)."""

    def __init__(self, n_modalities: int = 5, n_classes: int = 2, *, in_channels: Optional[int] = None,
                 out_channels: Optional[int] = None, precision: str = "bf16", checkpoint_decoder: bool = False):
        super().__init__()
        if in_channels is not None:
            n_modalities = in_channels
        if out_channels is not None:
            n_classes = out_channels
        if precision not in ("bf16", "fp32"):
            raise ValueError("precision must be 'bf16' or 'fp32'")
        self.n_modalities = n_modalities
        self.n_classes = n_classes
        self.init_features = 64
        self.precision = precision
        # decoder activation checkpointing (config 5; no reference equivalent)
        self.checkpoint_decoder = bool(checkpoint_decoder)
        f = self.init_features
        # construction order == reference order (same RNG consumption)
        self.inc = DoubleConv3D(n_modalities, f)
        self.down1 = Down3D(f, f * 2)
        self.down2 = Down3D(f * 2, f * 4)
        self.down3 = Down3D(f * 4, f * 8)
        self.down4 = Down3D(f * 8, f * 16)
        self.up1 = Up3D(f * 16, f * 8)
        self.up2 = Up3D(f * 8, f * 4)
        self.up3 = Up3D(f * 4, f * 2)
        self.up4 = Up3D(f * 2, f)
        self.outc = nn.Conv3d(f, n_classes, kernel_size=1)
        for m in self.modules():  # storage type of the sub-modules' stand-alone forward
            if isinstance(m, (DoubleConv3D, Down3D, Up3D)):
                m.precision = precision
        self._init_weights()
        self._engine: Optional[UNetEngine] = None

    def _init_weights(self):
        for m in self.modules():
            if isinstance(m, nn.Conv3d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm3d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    # -------------------------------------------------------------- engine plumbing
    def engine(self, full_sync: bool = True) -> UNetEngine:
        dev = self.outc.weight.device
        eng = self._engine
        if eng is None or eng.device != dev:
            eng = UNetEngine(self, dev, self.precision)
            self.__dict__["_engine"] = eng
        else:
            eng.sync_params(full=full_sync)
        eng.act_ckpt = self.checkpoint_decoder
        return eng

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_engine"] = None
        return st

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        eng = self.engine()
        if self.training and torch.is_grad_enabled():
            return _UNetFunction.apply(x, eng, *eng.params)
        if not self.training and torch.is_grad_enabled() and any(p.requires_grad for p in eng.params) \
                and x.requires_grad:
            raise NotImplementedError("eval-mode backward is not supported by the HIP engine")
        with torch.no_grad():
            return eng.forward(x, training=self.training)

    def predict(self, x):
        """eval + no_grad + sigmoid (models/unet3d.py:298-318); the sigmoid runs in the head
        kernel."""
        self.eval()
        with torch.no_grad():
            return self.engine().forward(x, training=False, act=1)

    def inference(self, x, threshold: float = 0.5):
        """Binary mask ``sigmoid(logits) > threshold`` as float (models/unet3d.py:320-344),
        thresholded in the head kernel."""
        self.eval()
        with torch.no_grad():
            return self.engine().forward(x, training=False, act=2, threshold=threshold)


def load_weights(model: UNet3D, checkpoint) -> UNet3D:
    """Load either checkpoint form the reference writes (script/validate_model.py:174-180,
    script/predict.py:139-145): a full ``save_checkpoint`` dict (``model_state_dict`` key) or
    a bare state dict (``best_model_epoch_*.pth``).  ``checkpoint``: a path or a loaded dict.
    Files are read with ``weights_only=True`` (nothing in them is executed)."""
    if isinstance(checkpoint, (str, bytes)) or hasattr(checkpoint, "__fspath__"):
        dev = next(model.parameters()).device
        checkpoint = torch.load(checkpoint, map_location=dev, weights_only=True)
    sd = checkpoint["model_state_dict"] if "model_state_dict" in checkpoint else checkpoint
    model.load_state_dict(sd)
    if model._engine is not None:
        model._engine.mark_dirty()
    return model
