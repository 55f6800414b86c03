"""Summarise the stem kernels' HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE) into the JSON bench.py reports as roofline.traffic (test tooling).

    python tests/kexp/stem_traffic.py <pmc dir> <out.json>
"""
import csv
import glob
import json
import os
import sys

csv.field_size_limit(sys.maxsize)
KERNELS = {"fwd": "stem_fwd_direct_kernel", "wgrad": "stem_wgrad_stream_kernel<4, 3, true",
           "reduce": "stem_wgrad_reduce_kernel"}


def means(path, counter):
    per = {k: {} for k in KERNELS}
    for fn in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            if r["Counter_Name"] != counter:
                continue
            for k, name in KERNELS.items():
                if name in r["Kernel_Name"]:
                    d = per[k]
                    d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v) if v else 0.0) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch, nf = means(os.path.join(d, "fetch"), "FETCH_SIZE")
    write, nw = means(os.path.join(d, "write"), "WRITE_SIZE")
    total = 2 * sum(fetch.values()) * 1024 + sum(write.values()) * 1024
    rec = {"shape": [2, 128, 128, 64], "kernels": list(KERNELS.values()),
           # the roofline kernel string bench.py reports for this pair (it uses the record only
           # when they match)
           "kernel": "stem conv3d 5->64 fwd + wgrad with the BN0 backward apply fused in (stem_fwd_direct_kernel<DENSE> + "
                     "stem_wgrad_stream_kernel<BN>)",
           "FETCH_SIZE_KB": fetch, "WRITE_SIZE_KB": write, "dispatches": {"fetch": nf, "write": nw},
           "correction": "FETCH_SIZE x2 (gfx950 reports half of a 16-B/lane streaming read, MI355X_MICROARCH.md "
                         "HBM section); WRITE_SIZE as reported",
           "traffic_bytes_per_pair": int(total),
           "source": "tests/kexp/pmc_stem_traffic.sh (separate --pmc passes over tests/bench_stem.py), "
                     "per-dispatch means"}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
