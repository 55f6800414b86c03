"""Diagnostic (not a test): the fp32 build's parity errors when some convs use bf16x3 instead of
bf16x6 (engine.set_fp32_conv_mode), on the golden cases: max train-logit error vs the
reference's fp32 logits (bar 1e-3), loss error (bar 1e-5) and the worst gradient rel-L2 as a
fraction of its bar (max(10 x the reference's own fp32 error, GRAD_RL2)); < 1 passes.
    python tests/diag_mixed_precision.py"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
import golden_util as gu  # noqa: E402

PRE_BN_BIAS = ("conv.0.bias", "conv.3.bias")
GRAD_RL2 = {"c16_bcedice": 5e-2, "cfg1_dice": 5e-3, "odd_bcedice": 5e-2, "c16_ncls2_dice": 5e-2, "zf_bcedice": 5e-2}
# self.convs order: enc0 c0, c1 (level 0), enc1 (1), enc2 (2), enc3 (3), enc4 (4), then dec
# blocks up1..up4 (levels 3, 2, 1, 0)
LEVEL = [0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 3, 3, 2, 2, 1, 1, 0, 0]
MIXES = {
    "x6 all": None,
    "x3 all": set(range(18)),
    "x3 levels 0-1 (not the stem)": {i for i in range(1, 18) if LEVEL[i] <= 1},
    "x3 level 1": {i for i in range(18) if LEVEL[i] == 1},
    "x3 levels 1-2": {i for i in range(18) if LEVEL[i] in (1, 2)},
    "x3 levels 2-4": {i for i in range(18) if LEVEL[i] >= 2},
    "x3 encoder 1-4": {i for i in range(2, 10)},
}


def run(name, mix):
    import pcms_amd  # noqa: F401
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.optim import FlatAdam
    from pcms_amd.utils.losses import BCEDiceLoss, DiceLoss
    g = gu.load(name)
    torch.manual_seed(0)
    m = UNet3D(n_modalities=5, n_classes=gu.CASES[name][0], precision="fp32").cuda()
    if mix:
        m.engine().set_fp32_conv_mode("x3", mix)
    crit = BCEDiceLoss() if gu.CASES[name][4] == "bce_dice" else DiceLoss()
    opt = FlatAdam(m, lr=gu.CASES[name][5], weight_decay=1e-5)
    x, y = gu.batch(name, 0)
    m.train()
    opt.zero_grad()
    lg = m(x.cuda())
    loss = crit(lg, y.cuda())
    loss.backward()
    le = float(np.abs(lg.detach().cpu().numpy() - g["logits_train"]).max())
    lo = abs(float(loss.detach()) - float(g["loss0"]))
    worst, wk = 0.0, ""
    for k, p in m.named_parameters():
        if k.endswith(PRE_BN_BIAS):
            continue
        got = gu.sampled(p.grad, g["g_stride__" + k]).astype(np.float64)
        r32, r64 = g["g__" + k].astype(np.float64), g["g64__" + k].astype(np.float64)
        nrm = np.linalg.norm(r64)
        if nrm == 0:
            continue
        frac = (np.linalg.norm(got - r64) / nrm) / max(10 * np.linalg.norm(r32 - r64) / nrm, GRAD_RL2[name])
        if frac > worst:
            worst, wk = frac, k
    return le, lo, worst, wk


def main():
    for label, mix in MIXES.items():
        print(f"== {label}", flush=True)
        for name in gu.CASES:
            le, lo, worst, wk = run(name, mix)
            print(f"   {name:16s} logits {le:.2e} ({le / 1e-3:.2f} of bar)  loss {lo:.1e}  worst grad {worst:.2f} of bar ({wk})",
                  flush=True)


if __name__ == "__main__":
    main()
