"""Print the last N kernels of a rocprofv3 kernel trace as a timeline
(start offset, duration, name).  python tools/trace_timeline.py CSV [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = None
prev_end = None
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t0 = s if t0 is None else t0
    gap = "" if prev_end is None else f"gap {(s - prev_end) / 1000:6.1f}"
    prev_end = e
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:7.1f} {gap:>11}  {r['Kernel_Name'][:70]}")
