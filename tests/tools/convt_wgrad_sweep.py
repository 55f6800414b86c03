"""ConvTranspose weight-gradient sweep (test tooling): pcms_convt_wgrad_bias at the engine's four
decoder shapes (N = 2), for each taps-per-workgroup setting (pcms_convt_wgrad_taps 8 / 4 / 2)
and workgroup target; HIP events around R back-to-back calls on one stream, median of 5.
Every setting's dw / db is checked against the TT = 8, target-512 result (fp32 sums in other
orders: max |diff| relative to max |dw| is printed).

    python tests/tools/convt_wgrad_sweep.py [--targets 256,512,1024] [--tts 8,4,2]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [((8, 8, 4), 1024, 512), ((16, 16, 8), 512, 256), ((32, 32, 16), 256, 128), ((64, 64, 32), 128, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--targets", default="256,512,1024")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tts", default="0,8,4,2")
    a = ap.parse_args()
    import pcms_amd  # noqa: F401
    from pcms_amd import _lib as L
    dev = "cuda"
    N = 2
    g = torch.Generator(device=dev).manual_seed(3)
    for Sin, cin, cout in SHAPES:
        Sout = tuple(2 * v for v in Sin)
        x = torch.randn(N, *Sin, cin, device=dev, generator=g).to(torch.bfloat16)
        dout = torch.randn(N, *Sout, cout, device=dev, generator=g).to(torch.bfloat16)
        ref = None
        for tt in [int(t) for t in a.tts.split(",")]:
            for target in [int(t) for t in a.targets.split(",")]:
                L.query("pcms_convt_wgrad_taps", tt)
                ws = torch.empty(L.query("pcms_convt_wgrad_ws_floats", N, *Sin, cin, cout, target), device=dev)
                bws = torch.empty(L.query("pcms_convt_wgrad_bias_ws_floats", 1, N, *Sin, cin, cout, target),
                                  device=dev)
                dw = torch.zeros(cin, cout, 2, 2, 2, device=dev)
                db = torch.zeros(cout, device=dev)

                def run():
                    L.call("pcms_convt_wgrad_bias", 1, x, dout, dw, db, ws, bws, N, *Sin, cin, cout, *Sout, target)
                run()
                torch.cuda.synchronize()
                one_dw, one_db = dw.clone(), db.clone()
                if ref is None:
                    ref = (one_dw, one_db)
                err_w = ((one_dw - ref[0]).abs().max() / ref[0].abs().max()).item()
                err_b = ((one_db - ref[1]).abs().max() / ref[1].abs().max()).item()
                ts = []
                for _ in range(5):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.reps):
                        run()
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1000 / a.reps)
                print(f"{cin}->{cout} {'x'.join(map(str, Sin))}  TT {tt}  target {target:5d}: "
                      f"{statistics.median(ts):7.1f} us   (dw rel {err_w:.1e}, db rel {err_b:.1e})", flush=True)
    L.query("pcms_convt_wgrad_taps", 0)


if __name__ == "__main__":
    main()
