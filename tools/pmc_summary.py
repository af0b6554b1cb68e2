#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc counter_collection.csv
files under the given directories (one row per kernel, torch/runtime kernels
dropped). usage: tools/pmc_summary.py DIR [DIR...]"""
import collections
import csv
import glob
import os
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
                if "at::" in n or "rocclr" in n:
                    continue
                agg[n.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for n, c in agg.items():
        print(n)
        for k in sorted(c):
            v = c[k]
            print(f"    {k:28s} {sum(v) / len(v):14.4g}  (n={len(v)})")


if __name__ == "__main__":
    main()
