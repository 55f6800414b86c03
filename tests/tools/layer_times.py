"""Per-launch timing of one training step at a BASELINE config (HIP events around every
library call the engine makes, median over the recorded steps), with FLOPs and the MFMA
fraction for the conv launches.  Diagnostic tool for profiles/ (not a test)."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

PEAK = 2.5e15


def flops(name, a):
    if name == "pcms_conv3_fwd":
        return 2 * 27 * (a[2] + a[4]) * a[17] * a[13] * a[14] * a[15] * a[16]
    if name == "pcms_conv3_wgrad":
        return 2 * 27 * (a[2] + a[4]) * a[12] * a[8] * a[9] * a[10] * a[11]
    if name == "pcms_conv3_fwd16":
        return 2 * 27 * (a[1] + a[3]) * a[17] * a[13] * a[14] * a[15] * a[16]
    if name == "pcms_conv3_fwd_bnin":
        return 2 * 27 * a[2] * a[13] * a[9] * a[10] * a[11] * a[12]
    if name == "pcms_conv3_wgrad_bnin":
        return 2 * 27 * a[2] * a[12] * a[8] * a[9] * a[10] * a[11]
    if name == "pcms_stem_fwd":
        return 2 * 27 * 5 * 64 * a[5] * a[6] * a[7] * a[8]
    if name == "pcms_stem_wgrad":
        return 2 * 27 * 5 * 64 * a[5] * a[6] * a[7] * a[8]
    if name in ("pcms_convt_fwd", "pcms_convt_wgrad", "pcms_convt_dgrad_ws"):
        return 2 * 8 * a[9] * a[10] * a[5] * a[6] * a[7] * a[8]
    if name == "pcms_convt_dgrad":
        return 2 * 8 * a[8] * a[9] * a[4] * a[5] * a[6] * a[7]
    if name == "pcms_convt_fwd_ws":
        return 2 * 8 * a[10] * a[11] * a[6] * a[7] * a[8] * a[9]
    if name == "pcms_convt_wgrad_bias":
        return 2 * 8 * a[11] * a[12] * a[7] * a[8] * a[9] * a[10]
    return 0


def desc(name, a):
    if name == "pcms_conv3_fwd":
        return f"{a[2]}+{a[4]}->{a[17]} {a[14]}x{a[15]}x{a[16]} sp{a[18]}" + (" dgrad" if a[6] is None else "")
    if name == "pcms_conv3_wgrad":
        return f"{a[2]}+{a[4]}->{a[12]} {a[9]}x{a[10]}x{a[11]}"
    if name == "pcms_conv3_fwd16":
        return (f"{'bn(' if a[4] is not None else ''}{a[1]}{')' if a[4] is not None else ''}+{a[3]}->{a[17]} "
                f"{a[14]}x{a[15]}x{a[16]} 16x16x32" + (" dgrad" if a[7] is None else ""))
    if name == "pcms_convt_dgrad":
        return f"{a[8]}->{a[9]} {a[5]}x{a[6]}x{a[7]}"
    if name == "pcms_conv3_fwd_bnin":
        return f"bn({a[2]})->{a[13]} {a[10]}x{a[11]}x{a[12]}"
    if name == "pcms_conv3_wgrad_bnin":
        return f"bn({a[2]})->{a[12]} {a[9]}x{a[10]}x{a[11]}"
    if name in ("pcms_convt_fwd", "pcms_convt_wgrad", "pcms_convt_dgrad_ws"):
        return f"{a[9]}->{a[10]} {a[6]}x{a[7]}x{a[8]}"
    if name == "pcms_convt_fwd_ws":
        return f"{a[10]}->{a[11]} {a[7]}x{a[8]}x{a[9]}"
    if name == "pcms_convt_wgrad_bias":
        return f"{a[11]}->{a[12]} {a[8]}x{a[9]}x{a[10]}"
    return ""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", default="128,128,64")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"],
                    help="fp32: the conv MFMA fraction counts the bf16x6 work (6 bf16 MFMA products per product)")
    ap.add_argument("--wgrad-target", type=int, default=0, help="engine.wgrad_target override")
    ap.add_argument("--split-target", type=int, default=0, help="engine.split_target override")
    ap.add_argument("--big-min-boxes", type=int, default=0, help="pcms_conv3_big_min_boxes override")
    ap.add_argument("--fwd-box-vol", type=int, default=0, help="pcms_conv3_fwd_box_vol override (256)")
    ap.add_argument("--convt-taps", type=int, default=0, help="pcms_convt_wgrad_taps override (8 / 4 / 2)")
    ap.add_argument("--hog", type=int, default=0,
                    help="K spinning workgroups (tests/kexp/libcuhog.so) holding K CUs on a side stream during every "
                         "recorded step: what an RCCL kernel beside the backward does to each launch")
    ap.add_argument("--clock", action="store_true",
                    help="bracket every launch with bench.ClockProbe stamps: the shader clock per launch and the MFMA "
                         "fraction at that clock (the stamps add a few us of launches between layers)")
    a = ap.parse_args()
    import pcms_amd  # noqa: F401
    from pcms_amd import engine as E
    from pcms_amd.synthetic import make_batch
    from pcms_amd.utils.trainer import Trainer
    spatial = tuple(int(v) for v in a.size.split(","))
    torch.manual_seed(0)
    tr = Trainer({"device": "cuda", "learning_rate": 1e-4, "batch_size": a.batch, "num_epochs": 1,
                  "loss": "bce_dice", "precision": a.precision})
    xf = 6 if a.precision == "fp32" else 1  # bf16 MFMA work per FLOP of the 3x3x3 convs
    if a.wgrad_target:
        tr.model.engine().wgrad_target = a.wgrad_target
    if a.split_target:
        tr.model.engine().split_target = a.split_target
    if a.fwd_box_vol:
        from pcms_amd import _lib as L
        L.query("pcms_conv3_fwd_box_vol", a.fwd_box_vol)
    if a.convt_taps:
        from pcms_amd import _lib as L
        L.query("pcms_convt_wgrad_taps", a.convt_taps)
    if a.big_min_boxes:
        from pcms_amd import _lib as L
        L.query("pcms_conv3_big_min_boxes", a.big_min_boxes)
    b = make_batch(a.batch, spatial, seed=1)
    batch = {"image": b["image"].cuda(), "label": b["label"].cuda()}
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    orig = E.call
    rec = []

    probe = None
    if a.clock:
        import bench
        probe = bench.ClockProbe()

    def timed(name, *args):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c0 = probe.stamp() if probe else None
        s.record()
        r = orig(name, *args)
        e.record()
        c1 = probe.stamp() if probe else None
        rec.append((name, args, s, e, c0, c1))
        return r
    mods = [m for k, m in sys.modules.items() if k.startswith("pcms_amd") and getattr(m, "call", None) is orig]
    for m in mods:
        m.call = timed
    def clk(c0, c1):
        if c0 is None:
            return None
        import bench
        v = list(bench.ClockProbe.mhz(c0, c1).values())
        return statistics.median(v) if v else None

    hog = side = sink = None
    if a.hog:
        import ctypes
        hog = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kexp", "libcuhog.so"))
        hog.cu_hog.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
        side = torch.cuda.Stream()
        sink = torch.zeros(64, dtype=torch.int32, device="cuda")
    per = []
    for _ in range(a.steps):
        rec.clear()
        if hog is not None:
            side.wait_stream(torch.cuda.current_stream())
            hog.cu_hog(a.hog, 30000.0, sink.data_ptr(), side.cuda_stream)
        tr.step(batch)
        torch.cuda.synchronize()
        per.append([(n, ar, s.elapsed_time(e) * 1e3, clk(c0, c1)) for n, ar, s, e, c0, c1 in rec])
    for m in mods:
        m.call = orig
    rows = []
    for i, (n, ar, _, _) in enumerate(per[0]):
        us = statistics.median(p[i][2] for p in per)
        f = flops(n, ar) * (xf if n.startswith("pcms_conv3") else 1)
        row = {"i": i, "name": n, "desc": desc(n, ar), "us": round(us, 1), "gflop": round(f / 1e9, 2),
               "mfma_frac": round(f / (us * 1e-6) / PEAK, 3) if f else None}
        if probe:
            mhz = statistics.median(p[i][3] for p in per if p[i][3] is not None)
            row["mhz"] = round(mhz)
            row["mfma_frac_at_clock"] = round(f / (us * 1e-6) / (PEAK * mhz / 2400.0), 3) if f else None
        rows.append(row)
    tot = sum(r["us"] for r in rows)
    by = {}
    for r in rows:
        by[r["name"]] = by.get(r["name"], 0) + r["us"]
    print(f"sum of launches {tot / 1e3:.2f} ms")
    for k, v in sorted(by.items(), key=lambda kv: -kv[1]):
        print(f"  {k:28s} {v / 1e3:7.3f} ms")
    for r in sorted(rows, key=lambda r: -r["us"])[:60]:
        print(f"{r['i']:4d} {r['name']:22s} {r['desc']:34s} {r['us']:8.1f} us  {r['gflop']:8.1f} GF  {r['mfma_frac']}"
              + (f"  {r['mhz']} MHz  {r['mfma_frac_at_clock']}" if probe else ""))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"batch": a.batch, "size": spatial, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
