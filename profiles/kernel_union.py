"""GPU busy time of a rocprofv3 --kernel-trace run: the union of every kernel's
[start, end) interval (kernels on several streams overlap), per kernel-name prefix
and in total, against the span from the first kernel start to the last end.
    python3 profiles/kernel_union.py <rocprofv3 -d directory>"""
import csv
import glob
import json
import os
import sys


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


def main(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if not rows:
        print(json.dumps({"error": "no kernel trace under " + d}))
        return
    groups = {}
    for name, s, e in rows:
        key = name.split("<")[0].split("(")[0].replace("void ", "").strip()
        groups.setdefault(key, []).append((s, e))
    first = min(s for _, s, _ in rows)
    last = max(e for _, _, e in rows)
    out = {"span_s": (last - first) * 1e-9, "busy_union_s": union([(s, e) for _, s, e in rows]) * 1e-9,
           "kernels": {k: {"launches": len(v), "busy_union_s": round(union(v) * 1e-9, 6),
                           "sum_s": round(sum(e - s for s, e in v) * 1e-9, 6)} for k, v in sorted(groups.items())}}
    out["busy_fraction_of_span"] = round(out["busy_union_s"] / out["span_s"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
