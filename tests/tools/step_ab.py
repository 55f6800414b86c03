"""In-step A/B of engine knobs on ONE box (test tooling): the bench workload (2 x 5x128x128x64,
BCEDice, Adam) stepped with each variant in turn, rounds interleaved in ABBA order so box
drift hits every variant alike; HIP events around K back-to-back steps, median over rounds.

    python tests/tools/step_ab.py [--rounds 4] [--steps 10] [--variants base,nobnin,...]

Variants: base (the defaults), nobnin (engine.fuse_bnin off), densewg (stem weight gradient
in the dense-column form), split256 / split512 (engine.split_target), x6sync / x6dma (the fp32
build's weight gradient staged synchronously / streamed by LDS-DMA; with --precision fp32),
wred1 / wred0 (the weight gradient's split rows summed in one launch / by the two-stage pair),
ctside (ConvT weight gradient on the side stream), poolsep / poolfused (engine.pool_bn_apply_fused off / on), nopack (the input pack skipped: the upper bound of folding it into the stem kernels), sideK (conv weight gradients of levels >= K on the side stream; side99 = never), wtN
(engine.wgrad_target = N), q:NAME=V (the library switch pcms_NAME set to V, restored after)."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--variants", default="base,nobnin,densewg")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    import pcms_amd  # noqa: F401
    from pcms_amd import _lib as L
    from pcms_amd.synthetic import make_batch
    from pcms_amd.utils.trainer import Trainer
    torch.manual_seed(0)
    tr = Trainer({"device": "cuda", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1,
                  "loss": "bce_dice", "precision": a.precision})
    eng = tr.model.engine()
    b = make_batch(2, (128, 128, 64), seed=1)
    batch = {"image": b["image"].cuda(), "label": b["label"].cuda()}
    dflt = {"fuse_bnin": eng.fuse_bnin, "split_target": eng.split_target, "side": eng.wgrad_side_min_level,
            "wt": eng.wgrad_target, "nopack": eng.ablate_skip_pack_input, "ctside": eng.convt_wgrad_side,
            "pool": eng.pool_bn_apply_fused}
    dense0 = L.query("pcms_stem_wgrad_dense", -1)
    x6dma0 = L.query("pcms_conv3_wgrad_x6_dma", -1)
    wred0 = L.query("pcms_conv3_wgrad_reduce_fused", -1)

    qsaved = {}

    def setup(v):
        for name, old in qsaved.items():
            L.query(name, old)
            eng.buf_key = None
        qsaved.clear()
        eng.fuse_bnin, eng.split_target = dflt["fuse_bnin"], dflt["split_target"]
        eng.wgrad_side_min_level = dflt["side"]
        eng.wgrad_target = dflt["wt"]
        eng.ablate_skip_pack_input = dflt["nopack"]
        eng.convt_wgrad_side = dflt["ctside"]
        eng.pool_bn_apply_fused = dflt["pool"]
        L.query("pcms_stem_wgrad_dense", dense0)
        L.query("pcms_conv3_wgrad_x6_dma", x6dma0)
        L.query("pcms_conv3_wgrad_reduce_fused", wred0)
        if v == "nobnin":
            eng.fuse_bnin = False
        elif v == "bnin":
            eng.fuse_bnin = True
        elif v in ("poolsep", "poolfused"):
            eng.pool_bn_apply_fused = v == "poolfused"
        elif v in ("ctside", "ctmain"):
            eng.convt_wgrad_side = v == "ctside"
        elif v == "nopack":
            eng.ablate_skip_pack_input = True
        elif v == "densewg":
            L.query("pcms_stem_wgrad_dense", 1)
        elif v == "tapswg":
            L.query("pcms_stem_wgrad_dense", 0)
        elif v in ("x6sync", "x6dma"):  # the fp32 build's weight-gradient box stream
            L.query("pcms_conv3_wgrad_x6_dma", int(v == "x6dma"))
        elif v in ("wred1", "wred0"):
            L.query("pcms_conv3_wgrad_reduce_fused", int(v == "wred1"))
        elif v.startswith("q:"):
            name, val = v[2:].split("=")
            qsaved["pcms_" + name] = L.query("pcms_" + name, int(val))
            eng.buf_key = None  # workspace sizes may follow the switch: re-lay out
        elif v.startswith("wt"):
            eng.wgrad_target = int(v[2:])
        elif v.startswith("side"):
            eng.wgrad_side_min_level = int(v[4:])
        elif v.startswith("split"):
            eng.split_target = int(v[5:])
        elif v != "base":
            raise SystemExit(f"unknown variant {v}")

    names = a.variants.split(",")
    res = {v: [] for v in names}
    for r in range(a.rounds):
        # ABBA order (odd rounds reversed): a box whose clock drifts over the run moves every
        # variant alike instead of favouring the one that always runs later in a round
        for v in (names if r % 2 == 0 else names[::-1]):
            setup(v)
            for _ in range(2):
                tr.step(batch)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.steps):
                tr.step(batch)
            e1.record()
            e1.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.steps)
        print(f"round {r}: " + "  ".join(f"{v} {res[v][-1]:.3f}" for v in names), flush=True)
    base = statistics.median(res[names[0]])
    for v in names:
        m = statistics.median(res[v])
        print(f"{v:10s} median {m:.3f} ms/step  ({m / base - 1:+.2%} vs {names[0]})  all {[round(x, 3) for x in res[v]]}",
              flush=True)


if __name__ == "__main__":
    main()
