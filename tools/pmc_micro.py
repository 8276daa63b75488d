"""PMC counters of a micro that launches its variants in order, each `per`
times (stream_v4: 3 warm-up + 50 timed launches): mean counter value per
launch for each variant, in launch order.
Usage: python tools/pmc_micro.py RUN_DIR [per] [names file]"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 53
    names = open(sys.argv[3]).read().split("\n") if len(sys.argv) > 3 else None
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        acc[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(acc)
    counters = sorted({c for v in acc.values() for c in v})
    print("variant " + " ".join(f"{c:>22s}" for c in counters))
    for v in range(len(ids) // per):
        sel = ids[v * per:(v + 1) * per]
        mean = {c: sum(acc[i][c] for i in sel) / len(sel) for c in counters}
        label = names[v] if names and v < len(names) else str(v)
        print(f"{label:30s} " + " ".join(f"{mean[c]:22.6g}" for c in counters))


if __name__ == "__main__":
    main()
