#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs (one directory per pass) for one kernel:
per-dispatch counter values averaged over the dispatches whose name matches."""
import csv
import glob
import os
import sys
from collections import defaultdict


def summarise(root, match):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if match not in r["Kernel_Name"]:
                continue
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), v in per.items():
            vals[c].append(v)
    return {c: sum(v) / len(v) for c, v in vals.items()}


if __name__ == "__main__":
    root, match = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "correlate"
    for c, v in sorted(summarise(root, match).items()):
        print("%-28s %16.1f" % (c, v))
