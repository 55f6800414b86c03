"""Per-kernel summary (name, calls, total/avg us, %) from a rocprofv3 kernel-trace
(``*_kernel_stats.csv`` or the rocpd ``*.db``), for committing under profiles/."""
import csv
import glob
import os
import sqlite3
import sys


def rows_from(path):
    if path.endswith(".csv"):
        return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(path))]
    c = sqlite3.connect(path)
    q = "select name, count(*), sum(end - start) from kernels group by name"
    return [(n, int(k), float(t)) for n, k, t in c.execute(q)]


def main(d, out=None, steps=None):
    paths = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True) or \
        glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    rows = sorted(rows_from(paths[0]), key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    lines = ["Name,Calls,TotalDurationNs,AverageNs,Percentage"]
    for n, k, t in rows:
        lines.append(f'"{n}",{k},{t:.0f},{t / k:.1f},{100 * t / tot:.2f}')
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(f"total {tot / 1e6:.2f} ms" + (f"  ({tot / 1e6 / int(steps):.2f} ms/step over {steps})" if steps else ""))
    for n, k, t in rows[:45]:
        print(f"{t / 1e6:8.3f} ms {k:6d} {t / k / 1e3:9.1f} us {100 * t / tot:5.1f}% {n[:100]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
