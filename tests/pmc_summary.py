"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean over dispatches).

    python tests/pmc_summary.py gpurun_out/pmcX [filter-substring]

Reads every */*counter_collection.csv under the given directories, keeps kernels whose
name contains the filter, and prints counter means plus derived figures (VALU per MFMA,
wait fractions, HBM bytes with the gfx950 FETCH_SIZE x2 correction).
"""
import collections
import csv
import glob
import os
import sys


def load(dirs, flt):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row["Kernel_Name"]
                    if flt and flt not in name:
                        continue
                    short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
                    vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    args = sys.argv[1:]
    flt = ""
    dirs = [a for a in args if os.path.isdir(a)]
    rest = [a for a in args if not os.path.isdir(a)]
    if rest:
        flt = rest[0]
    for k, cs in load(dirs, flt).items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"== {k}  (dispatches/counter: {max(len(v) for v in cs.values())})")
        for c in sorted(m):
            print(f"   {c:32s} {m[c]:.4g}")
        if "SQ_INSTS_VALU" in m and "SQ_INSTS_VALU_MFMA_BF16" in m and m["SQ_INSTS_VALU_MFMA_BF16"]:
            print(f"   -> VALU per MFMA {(m['SQ_INSTS_VALU'] - m['SQ_INSTS_VALU_MFMA_BF16']) / m['SQ_INSTS_VALU_MFMA_BF16']:.2f}")
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   -> {c}/WAVE_CYCLES {m[c] / m['SQ_WAVE_CYCLES']:.3f}")
        if "FETCH_SIZE" in m:
            print(f"   -> HBM read (FETCH_SIZE x2) {2 * m['FETCH_SIZE'] * 1024 / 1e6:.1f} MB")
        if "WRITE_SIZE" in m:
            print(f"   -> HBM write {m['WRITE_SIZE'] * 1024 / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
