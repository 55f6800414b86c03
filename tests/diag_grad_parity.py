"""Diagnostic (GPU): per-parameter gradient error of the fp32 engine vs the reference's fp64
truth, next to the reference fp32 CPU path's own error.  Prints one line per tensor.

    python tests/diag_grad_parity.py [case]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tests import golden_util as gu  # noqa: E402


def main(name):
    import pcms_amd
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.utils.losses import BCEDiceLoss, DiceLoss
    g = gu.load(name)
    ncls, n, spatial, lab, lk, lr = gu.CASES[name]
    torch.manual_seed(0)
    m = UNet3D(5, ncls, precision="fp32").cuda()
    crit = BCEDiceLoss() if lk == "bce_dice" else DiceLoss()
    x, y = gu.batch(name, 0)
    m.train()
    logits = m(x.cuda())
    loss = crit(logits, y.cuda())
    loss.backward()
    lg = logits.detach().cpu().numpy()
    print(f"{name}: logits err vs ref32 {np.abs(lg - g['logits_train']).max():.3e}  vs ref64 "
          f"{np.abs(lg - g['logits_train64']).max():.3e}  ref32-vs-64 "
          f"{np.abs(g['logits_train'] - g['logits_train64']).max():.3e}")
    print(f"  loss {float(loss.detach()):.8f} ref32 {float(g['loss0']):.8f} ref64 {float(g['loss0_64']):.8f}")
    for k, p in m.named_parameters():
        got = gu.sampled(p.grad, g["g_stride__" + k]).astype(np.float64)
        r32, r64 = g["g__" + k].astype(np.float64), g["g64__" + k].astype(np.float64)
        nrm = np.linalg.norm(r64) + 1e-30
        print(f"  {k:45s} scale {np.abs(r64).max():.2e} | us: max {np.abs(got - r64).max():.2e} "
              f"rl2 {np.linalg.norm(got - r64) / nrm:.2e} | ref32: max {np.abs(r32 - r64).max():.2e} "
              f"rl2 {np.linalg.norm(r32 - r64) / nrm:.2e}")


if __name__ == "__main__":
    for nm in (sys.argv[1:] or list(gu.CASES)):
        main(nm)
