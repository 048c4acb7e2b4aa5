#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/pass*_counter_collection.csv): per kernel, the
average of every counter per dispatch.  With --traffic INPUT_BYTES, also write
profiles/map_traffic.json for bench.py's roofline.traffic: HBM bytes per k_map launch =
2 x FETCH_SIZE (gfx950 tallies 128-B streaming reads at 64 B: MI355X_MICROARCH.md §HBM) + WRITE_SIZE,
both in KiB."""
import argparse
import collections
import csv
import glob
import json
import os


def load(pmc_dir, pattern="*counter_collection.csv"):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(pmc_dir, "**", pattern), recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def short(name):
    for k in ("k_map", "k_bucket_agg", "k_scatter", "k_tile_hist", "k_partition", "k_wc_write", "k_wc_len",
              "k_table_insert", "k_long", "k_gen", "k_make_sortrec"):
        if k in name:
            return k + ("<" + name.split("ILi")[1].split("E")[0] + ">" if "ILi" in name and k == "k_map" else "")
    return name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="gpurun_out/pmc")
    ap.add_argument("--traffic", type=int, default=0, help="input bytes per k_map launch")
    ap.add_argument("--out", default="profiles/map_traffic.json")
    ap.add_argument("--glob", default="*counter_collection.csv", help="CSV file pattern under --dir")
    ap.add_argument("--only", default="", help="print only kernels whose short name starts with this")
    a = ap.parse_args()
    per = load(a.dir, a.glob)
    rows = []
    for name, ctr in per.items():
        s = short(name)
        if not any(k in s for k in ("k_map", "k_bucket_agg", "k_scatter", "k_partition", "k_wc", "k_table")):
            continue
        avg = {c: sum(v) / len(v) for c, v in ctr.items()}
        rows.append((s, avg, max(len(v) for v in ctr.values())))
    for s, avg, n in rows:
        if a.only and not s.startswith(a.only):
            continue
        print(f"{s}  ({n} dispatch-counter rows)")
        for c in sorted(avg):
            print(f"    {c:28s} {avg[c]:.4g}")
    if a.traffic:
        km = [avg for s, avg, _ in rows if s.startswith("k_map")]
        if not km or "FETCH_SIZE" not in km[0] or "WRITE_SIZE" not in km[0]:
            raise SystemExit("need FETCH_SIZE and WRITE_SIZE rows for k_map")
        f, w = km[0]["FETCH_SIZE"], km[0]["WRITE_SIZE"]
        hbm = int((2 * f + w) * 1024)
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from mapreduce_rust_amd.native import kernel_source_sha
        doc = {"input_bytes": a.traffic, "hbm_bytes_per_launch": hbm, "kernel_src_sha": kernel_source_sha(),
               "fetch_size_kib": f, "write_size_kib": w,
               "rule": "2 x FETCH_SIZE + WRITE_SIZE (KiB); gfx950 FETCH_SIZE halves 128-B streaming reads"}
        json.dump(doc, open(a.out, "w"), indent=1)
        print("traffic", doc)


if __name__ == "__main__":
    main()
