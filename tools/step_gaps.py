#!/usr/bin/env python3
"""Host gaps (> 10 us) inside the last full bench step of a rocprofv3 kernel-trace CSV."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
km = [i for i, r in enumerate(rows) if "k_map" in r["Kernel_Name"]]
a, b = km[-2], km[-1]
t0 = prev = int(rows[a]["Start_Timestamp"])
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    g = (s - prev) / 1e3
    if g > 10 or "k_map" in r["Kernel_Name"]:
        print(f"{(s - t0) / 1e3:9.1f} gap {g:7.1f}  {r['Kernel_Name'][:60]}")
    prev = max(prev, e)
