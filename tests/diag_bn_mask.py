"""Diagnostic (GPU): compare the engine's last-BN pre-ReLU output (up4.conv.4) and its ReLU
mask against an fp64 CPU forward of the same module tree."""
import copy
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from tests import golden_util as gu  # noqa: E402


def ref_forward(m, x):
    """fp64 torch forward through the module containers; returns dict of BN outputs."""
    outs = {}

    def dconv(seq, h, tag):
        h = seq[0](h)
        outs[tag + ".y1"] = h
        h = seq[1](h)
        outs[tag + ".bn1"] = h
        h = F.relu(h)
        h = seq[3](h)
        outs[tag + ".y2"] = h
        h = seq[4](h)
        outs[tag + ".bn2"] = h
        return F.relu(h)

    x1 = dconv(m.inc.conv, x, "inc")
    skips = [x1]
    h = x1
    for i in range(1, 5):
        d = getattr(m, f"down{i}").maxpool_conv
        h = dconv(d[1].conv, d[0](h), f"down{i}")
        skips.append(h)
    for i, s in zip(range(1, 5), (skips[3], skips[2], skips[1], skips[0])):
        up = getattr(m, f"up{i}")
        u = up.up(h)
        dz, dy, dx = (s.shape[k] - u.shape[k] for k in (2, 3, 4))
        u = F.pad(u, [dx // 2, dx - dx // 2, dy // 2, dy - dy // 2, dz // 2, dz - dz // 2])
        h = dconv(up.conv.conv, torch.cat([s, u], 1), f"up{i}")
    return outs


def grad_check(name):
    """compare the engine's gradient buffers at up4 against fp64 autograd."""
    import pcms_amd
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.utils.losses import BCEDiceLoss, DiceLoss
    ncls, n, spatial, lab, lk, lr = gu.CASES[name]
    torch.manual_seed(0)
    m = UNet3D(5, ncls, precision="fp32")
    mref = copy.deepcopy(m).double().train()
    m = m.cuda().train()
    x, y = gu.batch(name, 0)
    crit = BCEDiceLoss() if lk == "bce_dice" else DiceLoss()
    logits = m(x.cuda())
    loss = crit(logits, y.cuda())
    loss.backward()
    torch.cuda.synchronize()
    outs = ref_forward(mref, x.double())
    bn2 = outs["up4.bn2"]
    bn2.retain_grad()
    h = F.relu(bn2)
    h.retain_grad()
    lref = F.conv3d(h, mref.outc.weight, mref.outc.bias)
    p = torch.sigmoid(lref).reshape(-1)
    t = y.double().reshape(-1)
    dice = 1 - (2 * (p * t).sum() + 1) / (p.sum() + t.sum() + 1)
    L = (0.5 * F.binary_cross_entropy_with_logits(lref, y.double()) + 0.5 * dice) if lk == "bce_dice" else dice
    L.backward()
    eng = m._engine
    b = eng.bufs
    S = b["S"]
    N = x.shape[0]
    gH = b["gH"].view(N, *S[0], -1).permute(0, 4, 1, 2, 3).double().cpu()
    print(f"{name}: gH err {(gH - h.grad).abs().max():.3e} scale {h.grad.abs().max():.3e}")
    db_ref = bn2.grad.sum((0, 2, 3, 4))
    g_ours = gH * (bn2 > 0)
    print(f"  sum(da*mask_ref) vs ref dbeta: {(g_ours.sum((0, 2, 3, 4)) - db_ref).abs().max():.3e}; "
          f"engine dbeta err {(m.up4.conv.conv[4].bias.grad.double().cpu() - db_ref).abs().max():.3e}; "
          f"ref-module dbeta err {(mref.up4.conv.conv[4].bias.grad - db_ref).abs().max():.3e} scale {db_ref.abs().max():.3e}")


def main(name):
    import pcms_amd
    from pcms_amd.models.unet3d import UNet3D
    ncls = gu.CASES[name][0]
    torch.manual_seed(0)
    m = UNet3D(5, ncls, precision="fp32")
    mref = copy.deepcopy(m).double()
    m = m.cuda()
    x, y = gu.batch(name, 0)
    m.train()
    with torch.no_grad():
        m(x.cuda())
    outs = ref_forward(mref.train(), x.double())
    eng = m._engine
    b = eng.bufs
    S = b["S"]
    for tag, buf, bn, lvl in (("up4", "d0_y2", eng.dec[3].b1, 0), ("up4", "d0_y1", eng.dec[3].b0, 0),
                              ("inc", "e0_y2", eng.enc[0].b1, 0)):
        key = tag + (".bn2" if buf.endswith("y2") else ".bn1")
        ykey = tag + (".y2" if buf.endswith("y2") else ".y1")
        N = x.shape[0]
        yy = b[buf].view(N, *S[lvl], -1).permute(0, 4, 1, 2, 3).double().cpu()
        sc, sh = bn.scale.double().cpu(), bn.shift.double().cpu()
        ours = yy * sc.view(1, -1, 1, 1, 1) + sh.view(1, -1, 1, 1, 1)
        ref = outs[key].detach()
        yref = outs[ykey].detach()
        flips = ((ours > 0) != (ref > 0)).sum().item()
        print(f"{name} {key}: y err {(yy - yref).abs().max():.3e} (scale {yref.abs().max():.2e})  "
              f"bn-out err {(ours - ref).abs().max():.3e}  mask flips {flips} / {ref.numel()}  "
              f"mean-shift/std max {(yref.mean((0, 2, 3, 4)).abs() / yref.std((0, 2, 3, 4))).max():.2e}")


if __name__ == "__main__":
    for nm in (sys.argv[1:] or ["c16_bcedice", "odd_bcedice"]):
        grad_check(nm)
