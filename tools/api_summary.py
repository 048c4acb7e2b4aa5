#!/usr/bin/env python3
"""Summary of a rocprofv3 runtime trace directory: total time per HIP API function and per kernel /
copy over the last bench step (from the last k_map launch on), longest first."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]


def rows(pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


kern = rows("*kernel_trace.csv")
t0 = max(int(r["Start_Timestamp"]) for r in kern if "k_map" in r["Kernel_Name"])
for name, pat, key in (("HIP API", "*hip_api_trace.csv", "Function"), ("kernels", "*kernel_trace.csv", "Kernel_Name"),
                       ("copies", "*memory_copy_trace.csv", "Direction")):
    tot = collections.Counter()
    cnt = collections.Counter()
    for r in rows(pat):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < t0:
            continue
        k = r.get(key, "?")[:80]
        tot[k] += (e - s) / 1e3
        cnt[k] += 1
    print(f"== {name} (us, from the last k_map launch)")
    for k, v in tot.most_common(25):
        print(f"{v:10.1f} {cnt[k]:5d}  {k}")
