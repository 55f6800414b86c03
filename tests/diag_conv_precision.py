"""Diagnostic (GPU): fp32 conv3 forward error vs fp64, ours vs torch CPU fp32."""
import math
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")


def main():
    import pcms_amd  # noqa
    from pcms_amd import _lib as L
    g = torch.Generator().manual_seed(0)
    for cin, S in ((64, (16, 16, 16)), (128, (16, 16, 16)), (512, (4, 4, 4))):
        N, cout = 2, 64
        x = torch.relu(torch.randn(N, cin, *S, generator=g))
        w = torch.randn(cout, cin, 3, 3, 3, generator=g) * math.sqrt(2.0 / (27 * cout))
        ref = F.conv3d(x.double(), w.double(), None, padding=1)
        cpu = F.conv3d(x, w, None, padding=1).double()
        wp = torch.empty(L.query("pcms_conv3_pack_elems", 0, cout, cin), device="cuda")
        L.call("pcms_conv3_pack", 0, w.cuda(), wp, cout, cin, 0)
        y = torch.empty(N, *S, cout, device="cuda")
        L.call("pcms_conv3_fwd", 0, x.permute(0, 2, 3, 4, 1).contiguous().cuda(), cin, None, 0, wp, None, y, None,
               cout, None, None, 0, N, *S, cout, 1)
        ours = y.cpu().permute(0, 4, 1, 2, 3).double()
        sc = ref.abs().max().item()
        print(f"cin {cin}: scale {sc:.3e}  ours max {(ours - ref).abs().max():.3e} rms "
              f"{(ours - ref).pow(2).mean().sqrt():.3e} | torch-cpu max {(cpu - ref).abs().max():.3e} rms "
              f"{(cpu - ref).pow(2).mean().sqrt():.3e}")


if __name__ == "__main__":
    main()
