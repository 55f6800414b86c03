"""A/B timing of the level-0 ConvTranspose forward (Cin 128, Cout 64, 2 x 64x64x32 input):
the persistent stream kernel vs the LDS kernel, alternated on one box (HIP events, median of
25 launches each, a GPU sleep before each launch so the host launch is not on the clock).
Diagnostic tool, not a test."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import pcms_amd  # noqa: E402,F401
from pcms_amd import _lib as L  # noqa: E402

N, Din, Hin, Win, cin, cout = 2, 64, 64, 32, 128, 64
x = torch.randn(N * Din * Hin * Win * cin, device="cuda").to(torch.bfloat16)
fp = torch.empty(L.query("pcms_convt_pack_elems", 1, cin, cout), dtype=torch.bfloat16, device="cuda")
L.call("pcms_convt_pack", 1, torch.randn(cin * cout * 8, device="cuda"), fp, cin, cout, 0)
b = torch.randn(cout, device="cuda")
out = torch.empty(N * 2 * Din * 2 * Hin * 2 * Win * cout, dtype=torch.bfloat16, device="cuda")
for on in (1, 0, 1, 0):
    L.query("pcms_convt_fwd_stream", on)
    ts = []
    for i in range(30):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(2000000)
        s.record()
        L.call("pcms_convt_fwd", 1, x, fp, b, out, N, Din, Hin, Win, cin, cout, 2 * Din, 2 * Hin, 2 * Win)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    print("stream" if on else "lds", round(statistics.median(ts[5:]), 1), "us", flush=True)
