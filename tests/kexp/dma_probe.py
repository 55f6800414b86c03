"""Drive tests/kexp/dma_probe.hip (test tooling): time each staging variant of the level-0
weight gradient's box stream (no MFMAs) and print us per launch and staged GB/s per CU.
    make -C tests/kexp libdmaprobe.so && python tests/kexp/dma_probe.py"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = {0: "product shape, 1 box in flight", 1: "2 boxes in flight", 2: "register loads + ds_write",
         3: "register loads, 2 in flight", 4: "L2-resident source", 5: "L2-resident, 2 in flight",
         8: "x halo as 128-B rows", 9: "128-B halo rows, 2 in flight", 16: "dy tile only", 17: "dy only, 2 in flight",
         32: "x halo only", 33: "halo only, 2 in flight", 20: "dy only, L2-resident", 36: "halo only, L2-resident",
         320: "MFMA phase alone (no staging)", 448: "LDS-fed MFMA phase alone", 384: "LDS reads alone",
         64: "staging + MFMA phase", 128: "staging + LDS reads", 192: "staging + LDS-fed MFMAs",
         576: "interleaved staging + MFMA phase", 704: "interleaved staging + LDS-fed MFMAs",
         66: "register staging + MFMA phase", 194: "register staging + LDS-fed MFMAs",
         1344: "zero-operand MFMA phase alone", 1088: "staging + zero-operand MFMAs",
         1600: "interleaved staging + zero-op MFMAs",
         2048: "SIMD-3 waves stage (no MFMAs)", 2112: "SIMD-3 stages, SIMDs 0-2 MFMA",
         2368: "SIMDs 0-2 MFMA alone", 2496: "SIMDs 0-2 LDS-fed MFMA alone", 2240: "SIMD-3 stages, 0-2 LDS-fed MFMA",
         4096: "16 waves stage", 4160: "16 waves: staging + MFMA phase", 4416: "16 waves: MFMA phase alone",
         4544: "16 waves: LDS-fed MFMA alone", 4288: "16 waves: staging + LDS-fed MFMA",
         8192: "blocked x: staging", 8193: "blocked x: 2 in flight", 8224: "blocked x: halo only",
         8228: "blocked x: halo only, L2-resident", 8256: "blocked x: staging + MFMA phase",
         8384: "blocked x: staging + LDS-fed MFMAs",
         16832: "LDS-fed MFMA alone, half the reads", 16576: "staging + LDS-fed MFMAs, half reads"}


def main():
    ex = ctypes.CDLL(os.path.join(HERE, "libdmaprobe.so"))
    N, D, H, W = 2, 128, 128, 64
    nvox = N * D * H * W
    x = torch.randn(nvox * 64, device="cuda").to(torch.bfloat16)
    dy = torch.randn(nvox * 64, device="cuda").to(torch.bfloat16)
    sink = torch.zeros(512, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    nbox = N * (D // 4) * (H // 8) * (W // 8)
    grid = 2 * nbox // 64
    sel = [int(v) for v in os.environ.get("FLAGS", "").split(",") if v]
    for F, name in NAMES.items():
        if sel and F not in sel:
            continue
        args = (F, ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(dy.data_ptr()), N, D, H, W,
                ctypes.c_void_p(sink.data_ptr()), st)
        rc = ex.probe_run(*args)
        assert rc == 0, (F, rc)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ex.probe_run(*args)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        us = sorted(ts)[2]
        # the clock the CUs ran at during the last launch: shader-clock ticks / 100 MHz ticks
        clk = (ctypes.c_ulonglong * (4 * grid))()
        mhz = float("nan")
        if ex.probe_clocks(clk, grid) == 0:
            c = [(clk[4 * i + 1] - clk[4 * i]) / max(1, clk[4 * i + 3] - clk[4 * i + 2]) * 100.0 for i in range(grid)]
            mhz = sorted(c)[len(c) // 2]
        wide = F & 8
        per_box = 0 if F & 256 else (0 if F & 32 else 256 * 128) + (0 if F & 16 else 600 * (128 if wide else 64))
        gbs = grid * 64 * per_box / (us * 1e-6) / 1e9
        print(f"F={F:5d} {name:36s} {us:8.1f} us  {per_box / 1024:5.1f} KB/box  {gbs / 256:6.1f} GB/s/CU  "
              f"{us / 64:5.2f} us/box  clock {mhz:6.0f} MHz", flush=True)


if __name__ == "__main__":
    main()
