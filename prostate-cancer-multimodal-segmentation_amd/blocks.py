"""Stand-alone execution of the U-Net sub-modules on the HIP kernels: ``DoubleConv3D(x)``,
``Down3D(x)`` and ``Up3D(x1, x2)`` called on their own (models/unet3d.py:42-55, 85-96,
124-158), as a reference user may do for feature extraction or block-level tests.

The hot path (``UNet3D.forward`` through ``engine.UNetEngine``) never comes here; this is
the same kernel library driven one block at a time:

* input NCDHW (any float dtype) -> NDHWC in the block's storage type, channels padded to a
  multiple of 8 (``pcms_pack_input``);
* Conv3d k3 p1 (``pcms_conv3_fwd``, weights packed per call), BatchNorm3d (train: batch
  statistics, running-stat update with the module's momentum / eps / num_batches_tracked;
  eval: running statistics), ReLU (``pcms_bn_relu``), MaxPool3d(2), ConvTranspose3d(k2, s2)
  with the symmetric pad of models/unet3d.py:143-151 folded into the output offsets and the
  channel concat [skip, up] (:156) read from two pointers;
* output NDHWC -> NCDHW fp32 (``pcms_unpack_output``).

Forward only: gradients flow through ``UNet3D`` as a whole (its autograd node runs the whole
HIP backward); a stand-alone call with an input that requires grad raises.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import BF16, F32, call, query

_T = {"bf16": (torch.bfloat16, BF16), "fp32": (torch.float32, F32)}


def _round8(c: int) -> int:
    return (c + 7) // 8 * 8


class _Runner:
    def __init__(self, precision: str, device: torch.device):
        if device.type != "cuda":
            raise RuntimeError("pcms_amd runs on a ROCm device only (no CPU path); move the module to 'cuda'")
        _lib.load()
        self.tdtype, self.code = _T[precision]
        self.dev = device

    def buf(self, n):
        return torch.empty(n, dtype=self.tdtype, device=self.dev)

    def pack(self, x: torch.Tensor):
        """NCDHW -> NDHWC storage tensor with round8(C) channels."""
        x = x.detach().to(self.dev, torch.float32).contiguous()
        N, C, D, H, W = x.shape
        cp = _round8(C)
        out = self.buf(N * D * H * W * cp)
        call("pcms_pack_input", self.code, x, out, N, C, D * H * W, cp)
        return out, cp

    def unpack(self, y, N, C, S):
        out = torch.empty((N, C) + tuple(S), dtype=torch.float32, device=self.dev)
        call("pcms_unpack_output", self.code, y, out, N, C, C, S[0] * S[1] * S[2])
        return out

    def conv_bn_relu(self, conv, bn, x0, c0, x1, c1, N, S, training):
        cout = conv.out_channels
        if cout % 64:
            raise ValueError("the HIP conv kernels need a multiple of 64 output channels")
        wpack = self.buf(query("pcms_conv3_pack_elems", self.code, cout, c0 + c1))
        call("pcms_conv3_pack", self.code, conv.weight.detach(), wpack, cout, conv.in_channels, 0)
        nvox = N * S[0] * S[1] * S[2]
        y = self.buf(nvox * cout)
        rows = query("pcms_conv3_fwd_rows", self.code, N, *S, c0, c1, cout)
        stats = torch.empty(rows * (cout * 2 + 1), dtype=torch.float32, device=self.dev)
        call("pcms_conv3_fwd", self.code, x0, c0, x1, c1, wpack, conv.bias, y, None, cout, None,
             stats if training else None, 0, N, *S, cout, 1)
        scale, shift, mean, invstd = (torch.empty(cout, device=self.dev) for _ in range(4))
        if training:
            if nvox <= 1:
                raise ValueError(f"Expected more than 1 value per channel when training, got input size "
                                 f"torch.Size([{N}, {cout}, {S[0]}, {S[1]}, {S[2]}])")
            ws = torch.empty(query("pcms_bn_ws_doubles", cout), dtype=torch.float64, device=self.dev)
            momentum = 0.1 if bn.momentum is None else float(bn.momentum)
            call("pcms_bn_finalize", stats, rows, cout, float(nvox), bn.weight, bn.bias, bn.running_mean,
                 bn.running_var, bn.num_batches_tracked, momentum, float(bn.eps), scale, shift, mean, invstd, ws)
        else:
            call("pcms_bn_eval_coeffs", bn.weight, bn.bias, bn.running_mean, bn.running_var, float(bn.eps), cout,
                 scale, shift)
        a = self.buf(nvox * cout)
        call("pcms_bn_relu", self.code, y, a, scale, shift, cout, nvox)
        return a, cout

    def double_conv(self, dc, x0, c0, x1, c1, N, S, training):
        seq = dc.conv
        a, c = self.conv_bn_relu(seq[0], seq[1], x0, c0, x1, c1, N, S, training)
        return self.conv_bn_relu(seq[3], seq[4], a, c, None, 0, N, S, training)


def _check_grad(*xs):
    if torch.is_grad_enabled() and any(isinstance(x, torch.Tensor) and x.requires_grad for x in xs):
        raise NotImplementedError("pcms_amd sub-modules run forward only; train through UNet3D.forward")


def _forward_only(fn):
    """Refuse inputs that require grad (checked under the caller's grad mode), then run
    ``fn`` under no_grad."""
    import functools

    @functools.wraps(fn)
    def wrapped(module, *xs):
        _check_grad(*xs)
        with torch.no_grad():
            return fn(module, *xs)
    return wrapped


def _runner(module, x):
    return _Runner(getattr(module, "precision", "bf16"), x.device)


@_forward_only
def double_conv_forward(dc, x: torch.Tensor) -> torch.Tensor:
    """DoubleConv3D.forward (models/unet3d.py:42-55)."""
    r = _runner(dc, x)
    N, _, D, H, W = x.shape
    xin, cp = r.pack(x)
    a, c = r.double_conv(dc, xin, cp, None, 0, N, (D, H, W), dc.training)
    return r.unpack(a, N, c, (D, H, W))


@_forward_only
def down_forward(down, x: torch.Tensor) -> torch.Tensor:
    """Down3D.forward: MaxPool3d(2) -> DoubleConv3D (models/unet3d.py:85-96)."""
    r = _runner(down, x)
    N, _, D, H, W = x.shape
    xin, cp = r.pack(x)
    S = (D // 2, H // 2, W // 2)
    if min(S) < 1:
        raise ValueError(f"input {tuple(x.shape)} is too small for MaxPool3d(2)")
    pooled = r.buf(N * S[0] * S[1] * S[2] * cp)
    call("pcms_maxpool_fwd", r.code, xin, pooled, N, D, H, W, cp)
    dc = down.maxpool_conv[1]
    a, c = r.double_conv(dc, pooled, cp, None, 0, N, S, down.training)
    return r.unpack(a, N, c, S)


@_forward_only
def up_forward(up, x1: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """Up3D.forward: ConvTranspose3d(k2, s2) on x1, symmetric pad to x2's size, cat([x2, x1]),
    DoubleConv3D (models/unet3d.py:124-158)."""
    r = _runner(up, x1)
    N, C1, Di, Hi, Wi = x1.shape
    C2, Do, Ho, Wo = x2.shape[1:]
    ct = up.up
    cout_t = ct.out_channels
    if C1 % 8 or C2 % 8 or cout_t % 8:
        raise ValueError("the HIP Up3D path needs channel counts that are multiples of 8")
    if min(Do - 2 * Di, Ho - 2 * Hi, Wo - 2 * Wi) < 0:
        raise ValueError("Up3D: the skip tensor must be at least twice the upsampled input's size")
    x1p, _ = r.pack(x1)
    x2p, _ = r.pack(x2)
    fpack = r.buf(query("pcms_convt_pack_elems", r.code, C1, cout_t))
    call("pcms_convt_pack", r.code, ct.weight.detach(), fpack, C1, cout_t, 0)
    u = r.buf(N * Do * Ho * Wo * cout_t)
    call("pcms_convt_fwd", r.code, x1p, fpack, ct.bias, u, N, Di, Hi, Wi, C1, cout_t, Do, Ho, Wo)
    a, c = r.double_conv(up.conv, x2p, C2, u, cout_t, N, (Do, Ho, Wo), up.training)
    return r.unpack(a, N, c, (Do, Ho, Wo))
