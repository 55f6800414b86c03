"""Average rocprofv3 PMC counters per dispatch for kernels matching a substring (test tooling).

    python tests/pmc_summary.py <run_counter_collection.csv> [...] --kernel conv3_fwd_big
"""
import argparse
import csv
import sys

csv.field_size_limit(sys.maxsize)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--kernel", required=True)
    a = ap.parse_args()
    for fn in a.files:
        per = {}
        for r in csv.DictReader(open(fn)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            d = per.setdefault(r["Counter_Name"], {})
            d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        for name, d in sorted(per.items()):
            vals = list(d.values())
            print(f"{name:32s} dispatches={len(vals):3d} mean={sum(vals) / len(vals):.4g}")


if __name__ == "__main__":
    main()
