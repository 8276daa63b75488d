"""Summarise rocprofv3 PMC passes written by tools/profile.sh: mean counter
value per dispatch for each kernel.  Usage: python tools/pmc_summary.py DIR"""
import collections
import csv
import os
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(\w+(<[^>]*>)?)\(", name)
    return m.group(1) if m else name


def summarise(d):
    out = collections.defaultdict(dict)
    for sub in sorted(os.listdir(d)):
        path = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            acc[(short(r["Kernel_Name"]), r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for (k, c), per in acc.items():
            out[k][c] = sum(per.values()) / len(per)
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    want = sys.argv[2:] or None
    for k, cs in sorted(res.items()):
        if want and not any(w in k for w in want):
            continue
        for c, v in sorted(cs.items()):
            print(f"{k:28s} {c:24s} {v:.5g}")
