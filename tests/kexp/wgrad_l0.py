"""bf16 weight gradient at one level (fresh-gradient store), 3 launches: the command the PMC
passes of tests/kexp/pmc_wgrad.sh profile (test tooling).  WGRAD_LEVEL=0 (64 -> 64 at
2 x 128x128x64, default), 1 (128 -> 128 at 2 x 64x64x32), 3 (512 -> 512 at 2 x 16x16x8)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pcms_amd  # noqa: E402,F401
from pcms_amd import _lib as L  # noqa: E402

lev = int(os.environ.get("WGRAD_LEVEL", "0"))
N, c0 = 2, 64 << lev
D, H, W = 128 >> lev, 128 >> lev, 64 >> lev
co = c0
x0 = torch.relu(torch.randn(N * D * H * W * c0, device="cuda")).to(torch.bfloat16)
dy = torch.randn(N * D * H * W * co, device="cuda").to(torch.bfloat16)
dw = torch.zeros(co * c0 * 27, device="cuda")
ws = torch.empty(L.query("pcms_conv3_wgrad_ws_floats", 1, N, D, H, W, c0, 0, co, 256), device="cuda")
for _ in range(3):
    L.call("pcms_conv3_wgrad", 1, x0, c0, None, 0, dy, dw, ws, N, D, H, W, co, c0, 256, 1)
torch.cuda.synchronize()
