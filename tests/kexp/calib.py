"""HBM calibration on the box (test tooling): sustained GB/s of write/read/copy shapes at the
stem's byte counts (268 MB output, 3 rotating buffers > 256 MiB Infinity Cache).

    python tests/kexp/calib.py
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libcalib.so"))
    for n in ("calib_write16", "calib_write_stemshape", "calib_read16", "calib_copy16"):
        getattr(lib, n).restype = ctypes.c_int
    nbytes = 2 * 128 * 128 * 64 * 128  # 268 MB
    bufs = [torch.empty(nbytes, dtype=torch.uint8, device="cuda") for _ in range(3)]
    src = [torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda") for _ in range(3)]
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    L = ctypes.c_long

    def run(name, fn, moved, reps=20):
        for i in range(3):
            assert fn(i) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fn(i % 3)
        e1.record()
        e1.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e-3
        print(f"{name:40s} {t * 1e6:8.1f} us  {moved / t / 1e9:7.0f} GB/s", flush=True)

    for g in (256, 1024, 2048, 8192):
        run(f"write16 grid {g}", lambda i, g=g: lib.calib_write16(P(bufs[i]), L(nbytes), g, st), nbytes)
    for g in (256, 512):
        run(f"write dword stem-shape grid {g}",
            lambda i, g=g: lib.calib_write_stemshape(P(bufs[i]), L(nbytes), g, 256, st), nbytes)
    for g in (256, 1024, 4096):
        run(f"read16 grid {g}", lambda i, g=g: lib.calib_read16(P(src[i]), L(nbytes), g, P(out), st), nbytes)
    for g in (1024, 4096):
        run(f"copy16 grid {g}", lambda i, g=g: lib.calib_copy16(P(src[i]), P(bufs[i]), L(nbytes), g, st),
            2 * nbytes)
    run("torch fill_ (268 MB)", lambda i: (bufs[i].fill_(i), 0)[1], nbytes)
    run("torch copy_ (268 MB)", lambda i: (bufs[i].copy_(src[i]), 0)[1], 2 * nbytes)


if __name__ == "__main__":
    main()
