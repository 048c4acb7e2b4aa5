#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 SQLite database (rocpd *_results.db): calls, total and
average duration, like --stats' kernel_stats.csv.  Usage: rocpd_stats.py DB [--csv OUT] [--skip N]
(--skip: ignore the first N dispatches of every kernel, e.g. warm-up)."""
import argparse
import collections
import csv
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv", default="")
    ap.add_argument("--skip", type=int, default=0)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    rows = db.execute(f"select {name_col}, start, end from kernels order by start").fetchall()
    per = collections.defaultdict(list)
    for n, s, e in rows:
        per[n].append(e - s)
    out = []
    for n, d in per.items():
        d = d[a.skip:] or d
        out.append((sum(d), n, len(d), sum(d) / len(d), min(d), max(d)))
    out.sort(reverse=True)
    tot = sum(o[0] for o in out) or 1
    w = csv.writer(open(a.csv, "w")) if a.csv else None
    if w:
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for t, n, c, avg, mn, mx in out:
        print(f"{t / 1e6:10.3f} ms  {c:5d} x {avg / 1e3:10.1f} us  {100 * t / tot:5.1f}%  {n[:110]}")
        if w:
            w.writerow([n, c, t, avg, 100 * t / tot, mn, mx])


if __name__ == "__main__":
    main()
