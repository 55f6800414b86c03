"""CPU restatement of the reference 3D U-Net hot path — TEST INFRASTRUCTURE ONLY.

See ``oracle/__init__.py``.  Everything here is plain PyTorch CPU fp32 in the
reference's NCDHW layout.  Parameters are a flat ``OrderedDict`` whose keys and
order are exactly the reference ``UNet3D.state_dict()`` keys.

Reference anchors (all paths relative to the reference repo root):

* layer table / widths ............ models/unet3d.py:177-225 (init_features=64 @190)
* DoubleConv3D ..................... models/unet3d.py:27-40 (conv k3 p1 -> BN -> ReLU, x2)
* Down3D ........................... models/unet3d.py:78-83 (MaxPool3d(2) -> DoubleConv)
* Up3D ............................. models/unet3d.py:120-158 (ConvT k2 s2, pad, cat[skip, up])
* _init_weights .................... models/unet3d.py:227-245
* forward .......................... models/unet3d.py:247-296
* predict / inference .............. models/unet3d.py:298-344
* DiceLoss ......................... utils/losses.py:44-92
* BCEDiceLoss ...................... utils/losses.py:124-152
* train step ....................... utils/trainer.py:179-195, Adam @113-117
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

BN_EPS = 1e-5        # nn.BatchNorm3d default (models/unet3d.py:31,37)
BN_MOMENTUM = 0.1    # nn.BatchNorm3d default
FEAT = 64            # init_features, models/unet3d.py:190


# --------------------------------------------------------------------------------------
# layer table
# --------------------------------------------------------------------------------------
def layer_table(n_modalities: int = 5, n_classes: int = 2) -> List[Tuple[str, str, int, int]]:
    """(kind, prefix, cin, cout) in module-construction order (models/unet3d.py:193-222).

    kind: 'conv3' Conv3d k3 p1, 'bn' BatchNorm3d, 'convT' ConvTranspose3d k2 s2,
    'conv1' the 1x1x1 output conv.
    """
    f = FEAT
    t: List[Tuple[str, str, int, int]] = []

    def dconv(prefix: str, cin: int, cout: int) -> None:
        t.append(("conv3", prefix + ".conv.0", cin, cout))
        t.append(("bn", prefix + ".conv.1", cout, cout))
        t.append(("conv3", prefix + ".conv.3", cout, cout))
        t.append(("bn", prefix + ".conv.4", cout, cout))

    dconv("inc", n_modalities, f)
    for i, (ci, co) in enumerate([(f, 2 * f), (2 * f, 4 * f), (4 * f, 8 * f), (8 * f, 16 * f)], 1):
        dconv(f"down{i}.maxpool_conv.1", ci, co)
    for i, (ci, co) in enumerate([(16 * f, 8 * f), (8 * f, 4 * f), (4 * f, 2 * f), (2 * f, f)], 1):
        t.append(("convT", f"up{i}.up", ci, ci // 2))
        dconv(f"up{i}.conv", ci, co)
    t.append(("conv1", "outc", f, n_classes))
    return t


def _default_conv_init(w: torch.Tensor, b: torch.Tensor) -> None:
    """torch _ConvNd.reset_parameters: kaiming_uniform(a=sqrt 5) + uniform bias."""
    torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    fan_in, _ = torch.nn.init._calculate_fan_in_and_fan_out(w)
    bound = 1.0 / math.sqrt(fan_in) if fan_in > 0 else 0.0
    torch.nn.init.uniform_(b, -bound, bound)


def init_params(n_modalities: int = 5, n_classes: int = 2) -> "OrderedDict[str, torch.Tensor]":
    """Parameters + buffers exactly as ``UNet3D(n_modalities, n_classes)`` builds them
    under the caller's RNG state (models/unet3d.py:177-245).

    RNG order: every conv / convT draws its default init at construction, then
    ``_init_weights`` re-draws every Conv3d weight with kaiming_normal(fan_out, relu)
    and zeroes its bias; ConvTranspose3d keeps the default init (the isinstance check
    at models/unet3d.py:234 matches Conv3d only); BN weight 1, bias 0.
    """
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    table = layer_table(n_modalities, n_classes)
    for kind, p, ci, co in table:  # construction
        if kind in ("conv3", "conv1"):
            k = 3 if kind == "conv3" else 1
            w = torch.empty(co, ci, k, k, k)
            b = torch.empty(co)
            _default_conv_init(w, b)
            sd[p + ".weight"], sd[p + ".bias"] = w, b
        elif kind == "convT":
            w = torch.empty(ci, co, 2, 2, 2)
            b = torch.empty(co)
            _default_conv_init(w, b)
            sd[p + ".weight"], sd[p + ".bias"] = w, b
        else:
            sd[p + ".weight"] = torch.ones(co)
            sd[p + ".bias"] = torch.zeros(co)
            sd[p + ".running_mean"] = torch.zeros(co)
            sd[p + ".running_var"] = torch.ones(co)
            sd[p + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
    for kind, p, ci, co in table:  # _init_weights, module order
        if kind in ("conv3", "conv1"):
            torch.nn.init.kaiming_normal_(sd[p + ".weight"], mode="fan_out", nonlinearity="relu")
            torch.nn.init.constant_(sd[p + ".bias"], 0.0)
    return sd


def param_keys(sd: Dict[str, torch.Tensor]) -> List[str]:
    """Trainable parameter keys in ``model.parameters()`` order (82 for the U-Net)."""
    return [k for k in sd if not k.endswith(("running_mean", "running_var", "num_batches_tracked"))]


# --------------------------------------------------------------------------------------
# forward
# --------------------------------------------------------------------------------------
def _dconv(sd, p: str, x: torch.Tensor, training: bool) -> torch.Tensor:
    for c, b in ((".conv.0", ".conv.1"), (".conv.3", ".conv.4")):
        x = F.conv3d(x, sd[p + c + ".weight"], sd[p + c + ".bias"], padding=1)
        if training:
            sd[p + b + ".num_batches_tracked"] += 1
        x = F.batch_norm(x, sd[p + b + ".running_mean"], sd[p + b + ".running_var"],
                         sd[p + b + ".weight"], sd[p + b + ".bias"], training, BN_MOMENTUM, BN_EPS)
        x = F.relu(x)
    return x


def _up(sd, p: str, x1: torch.Tensor, x2: torch.Tensor, training: bool) -> torch.Tensor:
    x1 = F.conv_transpose3d(x1, sd[p + ".up.weight"], sd[p + ".up.bias"], stride=2)
    dz, dy, dx = (x2.shape[i] - x1.shape[i] for i in (2, 3, 4))
    # symmetric pad, lo = diff // 2 (models/unet3d.py:143-151)
    x1 = F.pad(x1, [dx // 2, dx - dx // 2, dy // 2, dy - dy // 2, dz // 2, dz - dz // 2])
    return _dconv(sd, p + ".conv", torch.cat([x2, x1], dim=1), training)  # skip first (:156)


def forward(sd, x: torch.Tensor, training: bool = True) -> torch.Tensor:
    """UNet3D.forward (models/unet3d.py:247-296); BN buffers of ``sd`` update in place."""
    x1 = _dconv(sd, "inc", x, training)
    skips = [x1]
    h = x1
    for i in range(1, 5):
        h = F.max_pool3d(h, 2)
        h = _dconv(sd, f"down{i}.maxpool_conv.1", h, training)
        skips.append(h)
    h = skips[4]
    for i, s in zip(range(1, 5), (skips[3], skips[2], skips[1], skips[0])):
        h = _up(sd, f"up{i}", h, s, training)
    return F.conv3d(h, sd["outc.weight"], sd["outc.bias"])


def predict(sd, x: torch.Tensor) -> torch.Tensor:
    """models/unet3d.py:298-318 — eval-mode forward + sigmoid."""
    with torch.no_grad():
        return torch.sigmoid(forward(sd, x, training=False))


def inference(sd, x: torch.Tensor, threshold: float = 0.5) -> torch.Tensor:
    """models/unet3d.py:320-344 — strict ``>`` threshold on sigmoid probabilities."""
    return (predict(sd, x) > threshold).float()


# --------------------------------------------------------------------------------------
# losses
# --------------------------------------------------------------------------------------
def dice_loss(pred: torch.Tensor, target: torch.Tensor, smooth: float = 1.0) -> torch.Tensor:
    """utils/losses.py:44-92: global (whole-batch) soft Dice on sigmoid(pred)."""
    if pred.shape != target.shape:
        raise ValueError(f"shape mismatch: pred.shape={pred.shape}, target.shape={target.shape}")
    p = torch.sigmoid(pred).reshape(-1)
    t = target.reshape(-1)
    inter = (p * t).sum()
    return 1 - (2.0 * inter + smooth) / (p.sum() + t.sum() + smooth)


def bce_dice_loss(pred, target, bce_weight: float = 0.5, dice_weight: float = 0.5):
    """utils/losses.py:124-152: w_b * mean BCEWithLogits + w_d * Dice."""
    bce = F.binary_cross_entropy_with_logits(pred, target)
    return bce_weight * bce + dice_weight * dice_loss(pred, target)


# --------------------------------------------------------------------------------------
# train step
# --------------------------------------------------------------------------------------
class RefStep:
    """The per-batch step of utils/trainer.py:179-195 on a parameter dict.

    ``lr`` as configured (1e-4 in every reference script), Adam betas/eps defaults,
    coupled weight_decay 1e-5 (utils/trainer.py:113-117).
    """

    def __init__(self, sd, lr: float = 1e-4, loss: str = "bce_dice", weight_decay: float = 1e-5):
        self.sd = sd
        self.keys = param_keys(sd)
        for k in self.keys:
            sd[k].requires_grad_(True)
        self.opt = torch.optim.Adam([sd[k] for k in self.keys], lr=lr, weight_decay=weight_decay)
        self.loss_fn = bce_dice_loss if loss == "bce_dice" else dice_loss

    def forward_backward(self, image, label):
        """zero_grad -> forward -> loss -> backward; returns (loss, logits)."""
        self.opt.zero_grad()
        logits = forward(self.sd, image, training=True)
        loss = self.loss_fn(logits, label)
        loss.backward()
        return loss.detach(), logits.detach()

    def step(self, image, label) -> float:
        loss, _ = self.forward_backward(image, label)
        self.opt.step()
        return float(loss)


def dp_step_simulated(sd, shards, lr: float = 1e-4, loss: str = "bce_dice", opt=None):
    """CPU simulation of one data-parallel step over ``len(shards)`` replicas.

    Semantics = DistributedDataParallel(broadcast_buffers=True) around the reference
    step: every replica starts from rank 0's parameters AND BN buffers, runs forward +
    loss + backward on its own shard (per-replica BN statistics, per-replica global Dice,
    SURVEY H6), gradients are averaged, one Adam step is applied; the BN buffers kept are
    rank 0's.  ``opt`` (an Adam over ``sd``'s parameters) may be passed to keep
    optimizer state across calls.  Returns (mean loss, opt).
    """
    keys = param_keys(sd)
    for k in keys:
        sd[k].requires_grad_(True)
    if opt is None:
        opt = torch.optim.Adam([sd[k] for k in keys], lr=lr, weight_decay=1e-5)
    loss_fn = bce_dice_loss if loss == "bce_dice" else dice_loss
    grads = None
    losses = []
    rank0_buffers = None
    for r, (img, lab) in enumerate(shards):
        rep = OrderedDict((k, v.detach().clone()) for k, v in sd.items())
        for k in keys:
            rep[k].requires_grad_(True)
        out = forward(rep, img, training=True)
        l = loss_fn(out, lab)
        l.backward()
        losses.append(float(l))
        g = [rep[k].grad.clone() for k in keys]
        grads = g if grads is None else [a + b for a, b in zip(grads, g)]
        if r == 0:
            rank0_buffers = {k: v.detach().clone() for k, v in rep.items() if k not in keys}
    opt.zero_grad()
    for k, g in zip(keys, grads):
        sd[k].grad = g / len(shards)
    opt.step()
    with torch.no_grad():
        for k, v in rank0_buffers.items():
            sd[k].copy_(v)
    return sum(losses) / len(losses), opt
