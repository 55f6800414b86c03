"""Check of bench.ClockProbe (pcms_clock_probe) against in-kernel clocks: spin kernels whose
waves stamp their own (s_memtime, s_memrealtime) at start and end, bracketed by two probes.
Prints the probe's per-XCD clock next to the spinning waves' own clock per XCD, and the
spread of (memtime - memrealtime x f) over one probe's blocks of one XCD (a shared counter
per XCD reads the same offset on every CU)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import pcms_amd  # noqa: E402,F401
from pcms_amd import _lib as L  # noqa: E402


def main():
    probe = bench.ClockProbe()
    res = []
    for cycles in (2_000_000, 50_000_000, 400_000_000):
        nb = 512
        out = torch.zeros(5 * nb, dtype=torch.int64, device="cuda")
        a = probe.stamp()
        L.call("pcms_clock_spin", out, nb, cycles)
        z = probe.stamp()
        torch.cuda.synchronize()
        per_probe = bench.ClockProbe.mhz(a, z)
        rows = out.view(-1, 5).cpu().tolist()
        own = {}
        for t0, r0, t1, r1, x in rows:
            own.setdefault(int(x) & 0xff, []).append((t1 - t0) / max(r1 - r0, 1) * 100.0)
        own = {x: round(statistics.median(v), 1) for x, v in sorted(own.items())}
        # cycle-counter offsets: spread of (memtime - memrealtime x f) over one probe's stamps,
        # within one CU (should be ~0) and across the CUs of one XCD
        av = a.view(-1, 3).cpu().tolist()
        spread = {}
        for x in sorted(set(int(r[2]) & 0xff for r in av)):
            f = per_probe.get(x, 2000.0) / 100.0
            by_cu = {}
            for t, r, loc in av:
                if int(loc) & 0xff == x:
                    by_cu.setdefault(loc, []).append(t - r * f)
            within = max(max(v) - min(v) for v in by_cu.values())
            across = [statistics.median(v) for v in by_cu.values()]
            spread[x] = {"cus": len(by_cu), "within_cu": round(within), "across_cus": round(max(across) - min(across))}
        res.append({"cycles": cycles, "probe_mhz": per_probe, "spin_waves_mhz": own, "offset_spread_cycles": spread})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
