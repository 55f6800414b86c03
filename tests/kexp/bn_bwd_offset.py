"""Does the relative placement of two streamed level-0 tensors matter (test tooling)?
pcms_bn_relu_bwd (reduce over da and y, finalize, apply -> dy) at level-0 size (2 x 128x128x64
voxels, 64 channels, bf16) with da / y / dy carved from one allocation at y - da = dy - y =
268 MB + off, for several offsets; HIP events, median of 20 calls.

    python tests/kexp/bn_bwd_offset.py
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import pcms_amd  # noqa: F401
    from pcms_amd import _lib as L
    dev = "cuda"
    C, nvox = 64, 2 * 128 * 128 * 64
    nb = nvox * C * 2
    offs = [0, 256, 4096, 65536 + 256, 2 * 1024 * 1024 + 4096]
    raw = torch.empty(3 * nb + 3 * max(offs) + 4096, dtype=torch.uint8, device=dev)
    g = torch.Generator(device=dev).manual_seed(1)
    src_da = torch.randn(nvox * C, device=dev, generator=g).to(torch.bfloat16)
    src_y = torch.randn(nvox * C, device=dev, generator=g).to(torch.bfloat16)
    scale, shift = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    mean, invstd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    gam = torch.ones(C, device=dev)
    rows = L.query("pcms_bn_bwd_rows", 1, C, nvox)
    part = torch.empty(rows * C * 2, device=dev)
    coef = torch.empty(3 * C, device=dev)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    ws = torch.empty(L.query("pcms_bn_ws_doubles", C), dtype=torch.float64, device=dev)
    for rep in range(2):
        for off in offs:
            base = 0
            da = raw[base:base + nb].view(torch.bfloat16)
            y = raw[base + nb + off:base + 2 * nb + off].view(torch.bfloat16)
            dy = raw[base + 2 * nb + 2 * off:base + 3 * nb + 2 * off].view(torch.bfloat16)
            da.copy_(src_da)
            y.copy_(src_y)

            def run():
                L.call("pcms_bn_relu_bwd", 1, da, y, scale, shift, mean, invstd, gam, part, coef, dg, db, dy, C,
                       nvox, ws)
            run()
            torch.cuda.synchronize()
            ts = []
            for _ in range(20):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000)
            print(f"rep {rep} offset {off:8d} B: {statistics.median(ts):7.1f} us (min {min(ts):.1f})", flush=True)


if __name__ == "__main__":
    main()
