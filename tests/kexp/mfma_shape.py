"""Drive tests/kexp/mfma_shape.hip on the box (test tooling): both MFMA shapes, equal FLOPs,
every CU, back-to-back launches; time, shader clock (bench.ClockProbe), TFLOP/s."""
import ctypes
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def main():
    import bench
    import pcms_amd  # noqa: F401
    lib = ctypes.CDLL(os.path.join(HERE, "libmfmashape.so"))
    src = (torch.randn(16384 * 8, device="cuda") * 0.5).to(torch.bfloat16)
    wts = (torch.randn(16384 * 8, device="cuda") * 0.5).to(torch.bfloat16)
    out = torch.zeros(256 * 512, device="cuda")
    probe = bench.ClockProbe()
    st = torch.cuda.current_stream().cuda_stream
    steps32 = 27 * 200
    for rnd in range(3):
        for shape in (32, 16):
            steps = steps32 if shape == 32 else steps32 // 2
            fn = lambda: lib.mfma_shape(shape, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(wts.data_ptr()),  # noqa
                                        ctypes.c_void_p(out.data_ptr()), steps, 256, ctypes.c_void_p(st))
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a = probe.stamp()
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            z = probe.stamp()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            mhz = statistics.median(bench.ClockProbe.mhz(a, z).values())
            flop = 256 * 8 * steps32 * 8 * 2 * 32 * 32 * 16  # WGs x waves x steps x MFMAs x flop
            print(json.dumps({"round": rnd, "shape": shape, "us": round(us, 1), "mhz": round(mhz),
                              "tflops": round(flop / us / 1e6, 1),
                              "frac_at_clock": round(flop / us / 1e-6 / (2.5e15 * mhz / 2400), 3)}), flush=True)


if __name__ == "__main__":
    main()
