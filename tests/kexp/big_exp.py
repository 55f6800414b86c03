"""Big-box forward experiments on the box (test tooling): F=0 must equal the product kernel;
the other variants switch parts off (see big_exp.hip) to show what bounds the chunk loop."""
import ctypes
import math
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
NAMES = {0: "product", 1: "no halo HBM", 2: "B one line", 3: "no halo + B one line", 4: "no stores",
         7: "no halo/B/stores", 8: "no A reads", 15: "no halo/B/stores/A", 16: "no MFMA",
         23: "no halo/B/stores/MFMA", 32: "halo from 1 MiB (L2 hits)", 36: "halo L2 hits, no stores",
         64: "odd slots start half a box late", 68: "desync + no stores",
         128: "contiguous 1 KiB halo runs", 132: "contiguous halo, no stores",
         256: "output stores sc1 (drop from L2)", 512: "output stores nt"}


def main():
    import pcms_amd  # noqa
    from pcms_amd import _lib as L
    ex = ctypes.CDLL(os.path.join(HERE, "libbigexp.so"))
    ex.exp_big.restype = ctypes.c_int
    P = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    N, D, H, W = 2, 128, 128, 64
    nvox = N * D * H * W
    T = torch.bfloat16
    shapes = [tuple(int(v) for v in s.split(",")) for s in (sys.argv[1:] or ["64,0,64", "64,64,64", "128,0,64"])]
    for c0, c1, cout in shapes:
        cin = c0 + c1
        xs = [(torch.randn(nvox * c0, device="cuda").to(T), torch.randn(nvox * max(c1, 8), device="cuda").to(T))
              for _ in range(3)]
        y = torch.empty(nvox * cout, dtype=T, device="cuda")
        y2 = torch.empty_like(y)
        w = torch.randn(cout, cin, 27, device="cuda") / math.sqrt(27 * cin)
        wp = torch.empty(cin // 32 * 27 * cout * 32, dtype=T, device="cuda")
        L.call("pcms_conv3_pack", 1, w, wp, cout, cin, 0)
        bias = torch.randn(cout, device="cuda")
        stats = torch.zeros(256 * (2 * cout + 1), device="cuda")
        x0, x1 = xs[0]
        L.call("pcms_conv3_fwd", 1, x0, c0, x1 if c1 else None, c1, wp, bias, y, None, cout, None, stats, 0,
               N, D, H, W, cout, 1)
        rc = ex.exp_big(0, P(x0), c0, P(x1) if c1 else None, c1, P(wp), P(bias), P(y2), P(stats), N, D, H, W,
                        cout, 0, st())
        torch.cuda.synchronize()
        same = torch.equal(y.view(torch.int16), y2.view(torch.int16))
        print(f"== {c0}+{c1}->{cout}: F=0 rc {rc} equal to product: {same}", flush=True)
        flop = 2.0 * nvox * cout * cin * 27
        runs = [(int(f), 0) for f in os.environ.get("FLAGS", "").split(",") if f] or [(f, 0) for f in NAMES]
        runs += [(64, int(d, 0)) for d in os.environ.get("DELAYS", "").split(",") if d]
        for F, dly in runs:
            def run(i):
                a, b = xs[i % 3]
                return ex.exp_big(F, P(a), c0, P(b) if c1 else None, c1, P(wp), P(bias), P(y2), P(stats),
                                  N, D, H, W, cout, dly << 16, st())
            for i in range(3):
                run(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(20):
                run(i)
            e1.record()
            e1.synchronize()
            t = e0.elapsed_time(e1) / 20 * 1e-3
            label = NAMES[F] if not dly else f"delay (slot % {dly >> 8}) x {dly & 255} sleeps"
            print(f"   F={F:2d} {label:34s} {t * 1e6:8.1f} us  {flop / t / 1e12:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
