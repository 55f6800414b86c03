"""Per-step kernel table from a rocprofv3 --stats kernel_stats.csv (test tooling).

    python tests/tools/kstats.py <run_kernel_stats.csv> [steps=7] [top=40]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total {tot / 1e6 / steps:.3f} ms/step over {steps} steps")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"{float(r['TotalDurationNs']) / 1e6 / steps:7.3f} ms/step {int(r['Calls']) / steps:6.1f} calls "
              f"{float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:110]}")


if __name__ == "__main__":
    main()
