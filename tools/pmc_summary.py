#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs: per kernel (name substring), the mean of
each counter over its dispatches.  Not part of the product.

    python tools/pmc_summary.py KERNEL_SUBSTRING CSV|DIR [CSV|DIR ...]

A directory stands for every *counter_collection.csv below it (the passes of
tools/gpu_pmc.sh).
"""
import collections
import csv
import glob
import os
import sys


def main():
    sub, files = sys.argv[1], []
    for a in sys.argv[2:]:
        files += sorted(glob.glob(os.path.join(a, "**", "*counter_collection.csv"), recursive=True)) if os.path.isdir(a) else [a]
    acc = collections.defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if sub in row["Kernel_Name"]:
                    acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k in sorted(acc):
        v = acc[k]
        print(f"{k:28s} {sum(v) / len(v):.6g}   (n={len(v)})")


if __name__ == "__main__":
    main()
