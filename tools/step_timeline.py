#!/usr/bin/env python3
"""Timeline of the last bench step from a rocprofv3 kernel-trace CSV: start (us from the step's
k_map), gap to the previous kernel, duration, name."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
i0 = [i for i, r in enumerate(rows) if "k_map" in r["Kernel_Name"]][-1]
t0 = prev = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} +{(s - prev) / 1e3:7.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:90]}")
    prev = e
