"""Prints the last graph replay of a rocprofv3 kernel trace as a timeline: per kernel its
duration and the gap since the previous kernel ended (ktimeline.py <kernel_trace.csv> <kernels
per step>)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2])
last = rows[-n:]
prev = None
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:7.1f}  gap {gap:6.1f}  {r['Kernel_Name'][:70]}")
    prev = e
print(f"step span {(int(last[-1]['End_Timestamp']) - t0) / 1e3:.1f} us")
