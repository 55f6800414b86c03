"""Summarise a rocprofv3 kernel-trace database (test tooling, not product code).

    python tests/prof_summary.py gpurun_out/prof_xxx/run_results.db [--csv out.csv] [--shapes NAME]

Prints per-kernel calls / total / mean / min / max (us) with short names; ``--shapes``
breaks one kernel down by launch grid (grid_x, grid_y, grid_z, lds) to separate layers.
"""
import argparse
import re
import sqlite3


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^void ", "", name)
    return name[:70].replace(",", ";")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--shapes", default=None)
    ap.add_argument("--steps", type=float, default=None, help="divide totals by this many steps")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, lds_size from kernels").fetchall()
    agg = {}
    for name, dur, gx, gy, gz, lds in rows:
        k = short(name)
        e = agg.setdefault(k, [0, 0.0, 1e30, 0.0])
        e[0] += 1
        e[1] += dur
        e[2] = min(e[2], dur)
        e[3] = max(e[3], dur)
    tot = sum(e[1] for e in agg.values())
    lines = ["name,calls,total_us,mean_us,min_us,max_us,pct"]
    for k, (n, t, lo, hi) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        div = a.steps or 1.0
        lines.append(f"{k},{n},{t / 1e3 / div:.1f},{t / n / 1e3:.1f},{lo / 1e3:.1f},{hi / 1e3:.1f},{100 * t / tot:.2f}")
    print("\n".join(lines))
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("\n".join(lines) + "\n")
    if a.shapes:
        sh = {}
        for name, dur, gx, gy, gz, lds in rows:
            if a.shapes not in name:
                continue
            e = sh.setdefault((gx, gy, gz, lds), [0, 0.0])
            e[0] += 1
            e[1] += dur
        print(f"\n{a.shapes}: grid_x,grid_y,grid_z,lds -> calls, mean_us")
        for k, (n, t) in sorted(sh.items(), key=lambda kv: -kv[1][1]):
            print(k, n, f"{t / n / 1e3:.1f}")


if __name__ == "__main__":
    main()
