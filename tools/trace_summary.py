#!/usr/bin/env python3
"""Per-launch durations of the dominant kernels from a rocprofv3 kernel trace (CSV): every launch,
and the average over the last N launches of each (the timed bench steps; the first launches are the
cold warm-up and any capacity rerun)."""
import collections
import csv
import sys

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 3
d = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    for k in ("k_map<", "k_bucket_agg<", "k_scatter<", "k_wc_write", "k_partition"):
        if k in n:
            d[k.rstrip("<")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in d.items():
    tail = v[-last:] if k in ("k_map", "k_bucket_agg") else v
    print(f"{k:14s} launches {len(v):3d}  all(ms) {' '.join(f'{x:.3f}' for x in v[:12])}{' ...' if len(v) > 12 else ''}")
    if k in ("k_map", "k_bucket_agg"):
        print(f"{'':14s} average of the last {len(tail)} (timed steps): {sum(tail) / len(tail):.3f} ms")
