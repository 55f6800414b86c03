"""Deep-level weight gradients (levels 3-4 of config 2) under the tap-group plan (TG, the
product: grids of <= 64 boxes split their taps over two workgroups) and the voxel-split plan
(pcms_conv3_wgrad_tg_maxbox(0)) at two workgroup targets; HIP events, median of 20, clock
(test tooling).  Usage: python tests/tools/wgrad_deep_ab.py"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # (N, D, H, W, c0, c1, Cout)
    (2, 16, 16, 8, 512, 0, 512), (2, 16, 16, 8, 512, 512, 512), (2, 16, 16, 8, 256, 0, 512),
    (2, 8, 8, 4, 1024, 0, 1024), (2, 8, 8, 4, 512, 0, 1024),
]


def main():
    import pcms_amd  # noqa: F401
    import bench
    from pcms_amd import _lib as L
    probe = bench.ClockProbe()
    T = torch.bfloat16
    for (N, D, H, W, c0, c1, co) in SHAPES:
        nvox = N * D * H * W
        cin = c0 + c1
        x0 = torch.randn(nvox * c0, device="cuda").to(T)
        x1 = torch.randn(nvox * max(c1, 8), device="cuda").to(T)
        dy = torch.randn(nvox * co, device="cuda").to(T)
        dw = torch.zeros(co * cin * 27, device="cuda")
        for tg, target in ((64, 256), (0, 256), (0, 512)):
            old = L.query("pcms_conv3_wgrad_tg_maxbox", tg)
            ws = torch.empty(max(1, L.query("pcms_conv3_wgrad_ws_floats", 1, N, D, H, W, c0, c1, co, target)),
                             device="cuda")

            def run():
                L.call("pcms_conv3_wgrad", 1, x0, c0, x1 if c1 else None, c1, dy, dw, ws, N, D, H, W, co, cin,
                       target, 1)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            k0 = probe.stamp()
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            k1 = probe.stamp()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            mhz = statistics.median(bench.ClockProbe.mhz(k0, k1).values())
            nspl = ws.numel() // (27 * co * cin) if ws.numel() > 1 else 1
            print(json.dumps({"shape": f"{c0}+{c1}->{co} {N}x{D}x{H}x{W}", "tg_maxbox": tg, "target": target,
                              "splits": nspl, "us": round(us, 1), "mhz": round(mhz)}), flush=True)
            L.query("pcms_conv3_wgrad_tg_maxbox", old)


if __name__ == "__main__":
    main()
