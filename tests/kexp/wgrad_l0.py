"""Level-0 bf16 weight gradient (64 -> 64 at 2 x 128x128x64, fresh-gradient store), 3 launches:
the command the PMC passes of tests/kexp/pmc_wgrad.sh profile (test tooling)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pcms_amd  # noqa: E402,F401
from pcms_amd import _lib as L  # noqa: E402

N, D, H, W, c0, co = 2, 128, 128, 64, 64, 64
x0 = torch.relu(torch.randn(N * D * H * W * c0, device="cuda")).to(torch.bfloat16)
dy = torch.randn(N * D * H * W * co, device="cuda").to(torch.bfloat16)
dw = torch.zeros(co * c0 * 27, device="cuda")
ws = torch.empty(L.query("pcms_conv3_wgrad_ws_floats", 1, N, D, H, W, c0, 0, co, 256), device="cuda")
for _ in range(3):
    L.call("pcms_conv3_wgrad", 1, x0, c0, None, 0, dy, dw, ws, N, D, H, W, co, c0, 256, 1)
torch.cuda.synchronize()
