#!/usr/bin/env python3
"""Per-dispatch means of rocprofv3 --pmc counter CSVs, for the dispatches whose kernel name
matches a pattern:  python scripts/pmc_summary.py DIR [DIR ...] --kernel gemm"""
import argparse
import collections
import csv
import glob
import os


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}, 0
    acc = collections.defaultdict(float)
    disp = set()
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            if pat and pat not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    n = max(1, len(disp))
    return {k: v / n for k, v in acc.items()}, len(disp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    for d in a.dirs:
        c, n = load(d, a.kernel)
        print(f"## {d} ({n} dispatches)")
        for k in sorted(c):
            print(f"  {k:32s} {c[k]:16.4g}")


if __name__ == "__main__":
    main()
