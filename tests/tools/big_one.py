"""One big-box conv shape launched `reps` times (test tooling, for rocprofv3 --pmc passes):
python tests/tools/big_one.py [shape index] [reps]; PCMS_LIB selects a variant library."""
import math
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tests.tools.big_abl import SHAPES  # noqa: E402


def main():
    import pcms_amd  # noqa: F401
    from pcms_amd import _lib as L
    si = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    N, D, H, W, c0, c1, cout = SHAPES[si]
    nvox = N * D * H * W
    cin = c0 + c1
    T = torch.bfloat16
    a = torch.randn(nvox * c0, device="cuda").to(T)
    b = torch.randn(nvox * max(c1, 8), device="cuda").to(T)
    y = torch.empty(nvox * cout, dtype=T, device="cuda")
    w = torch.randn(cout, cin, 27, device="cuda") / math.sqrt(27 * cin)
    wp = torch.empty(L.query("pcms_conv3_pack_elems", 1, cout, cin), dtype=T, device="cuda")
    L.call("pcms_conv3_pack", 1, w, wp, cout, cin, 0)
    bias = torch.randn(cout, device="cuda")
    stats = torch.zeros(L.query("pcms_conv3_fwd_rows", 1, N, D, H, W, c0, c1, cout) * (2 * cout + 1) + 1024,
                        device="cuda")
    for _ in range(reps):
        L.call("pcms_conv3_fwd", 1, a, c0, b if c1 else None, c1, wp, bias, y, None, cout, None, stats, 0,
               N, D, H, W, cout, 1)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
