"""One weight-gradient shape launched `reps` times (test tooling for rocprofv3 --pmc passes).
Usage: python tests/tools/wgrad_one.py SHAPE_INDEX REPS   (tests/tools/wgrad_abl.py SHAPES)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.tools.wgrad_abl import SHAPES  # noqa: E402


def main():
    i, reps = int(sys.argv[1]), int(sys.argv[2])
    import pcms_amd  # noqa: F401
    from pcms_amd import _lib as L
    N, D, H, W, c0, c1, co = SHAPES[i]
    nvox = N * D * H * W
    T = torch.bfloat16
    x0 = torch.randn(nvox * c0, device="cuda").to(T)
    x1 = torch.randn(nvox * max(c1, 8), device="cuda").to(T)
    dy = torch.randn(nvox * co, device="cuda").to(T)
    dw = torch.zeros(co * (c0 + c1) * 27, device="cuda")
    ws = torch.empty(max(1, L.query("pcms_conv3_wgrad_ws_floats", 1, N, D, H, W, c0, c1, co, 256)), device="cuda")
    for _ in range(reps):
        L.call("pcms_conv3_wgrad", 1, x0, c0, x1 if c1 else None, c1, dy, dw, ws, N, D, H, W, co, c0 + c1, 256, 1)
    torch.cuda.synchronize()
    print("ok", SHAPES[i])


if __name__ == "__main__":
    main()
