#!/usr/bin/env python3
"""Per-kernel PMC counter summary of a rocprofv3 --pmc run directory (all *counter_collection.csv).

usage: python scripts/pmc_summary.py gpurun_out/pmc [kernel-substring ...]
Prints, per kernel name (short) and counter, the mean over dispatches.
"""
import collections
import csv
import glob
import os
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n.replace("void ", "").replace("orion::", "")[:48]


def main():
    d = sys.argv[1]
    pats = sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            if pats and not any(p in k for p in pats):
                continue
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(acc):
        print(k)
        for c in sorted(acc[k]):
            v = acc[k][c]
            print(f"   {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")


if __name__ == "__main__":
    main()
