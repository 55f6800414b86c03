"""Summarise rocprofv3 --pmc passes (pmc_big.sh output): per counter, the median over the
dispatches of the kernel whose name contains argv[2], for each directory prefix argv[1]*."""
import csv
import glob
import statistics
import sys


def table(prefix, kname):
    vals = {}
    for f in sorted(glob.glob(f"{prefix}_p*/pmc_counter_collection.csv")):
        per = {}
        for r in csv.DictReader(open(f)):
            if kname not in r["Kernel_Name"]:
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        by = {}
        for (d, c), v in per.items():
            by.setdefault(c, []).append(v)
        for c, v in by.items():
            vals[c] = statistics.median(v)
    return vals


if __name__ == "__main__":
    k = sys.argv[2] if len(sys.argv) > 2 else "conv3_fwd_big"
    tabs = {p: table(p, k) for p in sys.argv[1].split(",")}
    names = sorted(set().union(*[set(t) for t in tabs.values()]))
    print("counter".ljust(40) + "".join(p.split("/")[-1][-22:].rjust(24) for p in tabs))
    for c in names:
        print(c.ljust(40) + "".join(f"{tabs[p].get(c, float('nan')):24.4g}" for p in tabs))
