"""Deep-level conv weight-gradient timing sweep (diagnostic, not a test): pcms_conv3_wgrad at
the level-2..4 shapes of config 2 for several workgroup targets (the split count follows),
fresh-gradient store mode, HIP events around each call (median of 20).
    python tests/tools/wgrad_sweep.py [--targets 128,256,512,1024]"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # (N, D, H, W, c0, c1, Cout)
    (2, 32, 32, 16, 256, 256, 256), (2, 32, 32, 16, 256, 0, 256),
    (2, 16, 16, 8, 512, 512, 512), (2, 16, 16, 8, 512, 0, 512), (2, 16, 16, 8, 256, 0, 512),
    (2, 8, 8, 4, 1024, 0, 1024), (2, 8, 8, 4, 512, 0, 1024),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--targets", default="128,256,512,1024")
    a = ap.parse_args()
    import pcms_amd  # noqa: F401
    from pcms_amd import _lib as L
    for N, D, H, W, c0, c1, co in SHAPES:
        cin = c0 + c1
        x0 = torch.randn(N * D * H * W * c0, device="cuda").to(torch.bfloat16)
        x1 = torch.randn(N * D * H * W * max(c1, 8), device="cuda").to(torch.bfloat16)
        dy = torch.randn(N * D * H * W * co, device="cuda").to(torch.bfloat16)
        dw = torch.zeros(co * cin * 27, device="cuda")
        line = f"{c0}+{c1}->{co} {D}x{H}x{W}:"
        for tg in (int(v) for v in a.targets.split(",")):
            ws = torch.empty(max(1, L.query("pcms_conv3_wgrad_ws_floats", 1, N, D, H, W, c0, c1, co, tg)),
                             device="cuda")
            ts = []
            for i in range(25):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                L.call("pcms_conv3_wgrad", 1, x0, c0, x1 if c1 else None, c1, dy, dw, ws, N, D, H, W, co, cin,
                       tg, 1)
                e.record()
                torch.cuda.synchronize()
                if i >= 5:
                    ts.append(s.elapsed_time(e) * 1e3)
            nspl = ws.numel() // (27 * co * cin) if ws.numel() > 1 else 1
            line += f"  t{tg}: {statistics.median(ts):6.1f} us (splits {nspl})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
