#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (gpurun_out/pmc/pass*_counter_collection.csv): per kernel, the
average of every counter per dispatch.  With --traffic INPUT_BYTES, also write
profiles/map_traffic.json for bench.py's roofline.traffic: HBM bytes per k_map launch =
2 x FETCH_SIZE (gfx950 tallies 128-B streaming reads at 64 B: MI355X_MICROARCH.md §HBM) + WRITE_SIZE,
both in KiB.
With --stages INPUT_BYTES, also write profiles/stage_traffic.json: HBM bytes per job (per bench step)
of each stage of the job -- map, aggregate, sort, format -- and of the whole job (every dispatch from
the first k_map launch on, fills / copies / scans included), 2 x FETCH_SIZE + WRITE_SIZE for every
kernel (the gfx950 factor is exact for 128-B streaming reads, an upper bound for narrower ones)."""
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


STAGES = {  # stage -> kernel-name fragments (libmrgpu.so kernels; anything else counts in the whole job only)
    "map": ("k_map<",),
    "aggregate": ("k_bucket_agg", "k_partition", "k_table_", "k_long_", "k_w", "k_flush"),
    "sort": ("k_make_sortrec", "k_msd_", "k_radix", "k_fix_runs", "k_sort"),
    "format": ("k_wc_len", "k_wc_write", "k_part_off", "k_total", "k_idx_"),
}


def stage_of(name):
    base = name.replace("(anonymous namespace)::", "").replace("void ", "")
    for st, frags in STAGES.items():
        for f in frags:
            if base.startswith(f) and not (f == "k_w" and base.startswith("k_wc_")):
                return st
    return None


def job_bytes(pmc_dir, pattern="*counter_collection.csv"):
    """Per counter: {stage: summed value over the job dispatches, '_job': all job dispatches}, and the
    number of jobs (k_map dispatches).  Job dispatches = from the first k_map dispatch on."""
    out = {}
    n_jobs = 0
    for f in sorted(glob.glob(os.path.join(pmc_dir, "**", pattern), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        first = min((int(r["Dispatch_Id"]) for r in rows if "k_map<" in r["Kernel_Name"]), default=None)
        if first is None:
            continue
        maps = {int(r["Dispatch_Id"]) for r in rows if "k_map<" in r["Kernel_Name"]}
        n_jobs = max(n_jobs, len(maps))
        for r in rows:
            if int(r["Dispatch_Id"]) < first:
                continue
            c = out.setdefault(r["Counter_Name"], collections.defaultdict(float))
            v = float(r["Counter_Value"])
            c["_job"] += v
            st = stage_of(r["Kernel_Name"])
            if st:
                c[st] += v
    return out, n_jobs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="gpurun_out/pmc")
    ap.add_argument("--traffic", type=int, default=0, help="input bytes per k_map launch")
    ap.add_argument("--out", default="profiles/map_traffic.json")
    ap.add_argument("--glob", default="*counter_collection.csv", help="CSV file pattern under --dir")
    ap.add_argument("--only", default="", help="print only kernels whose short name starts with this")
    ap.add_argument("--stages", type=int, default=0, help="input bytes per job: write --stages-out")
    ap.add_argument("--stages-out", default="profiles/stage_traffic.json")
    ap.add_argument("--workload", default="C3", help="label stored with --stages")
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
    if a.stages:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from mapreduce_rust_amd.native import kernel_source_sha
        jb, n_jobs = job_bytes(a.dir, a.glob)
        if "FETCH_SIZE" not in jb or "WRITE_SIZE" not in jb or not n_jobs:
            raise SystemExit("need FETCH_SIZE and WRITE_SIZE passes with k_map dispatches")
        keys = list(STAGES) + ["_job"]
        per = {k: int((2 * jb["FETCH_SIZE"].get(k, 0.0) + jb["WRITE_SIZE"].get(k, 0.0)) * 1024 / n_jobs) for k in keys}
        doc = {"input_bytes": a.stages, "workload": a.workload, "kernel_src_sha": kernel_source_sha(),
               "jobs": n_jobs, "stage_hbm_bytes": {k: per[k] for k in STAGES}, "job_hbm_bytes": per["_job"],
               "fetch_kib_per_job": {k: jb["FETCH_SIZE"].get(k, 0.0) / n_jobs for k in keys},
               "write_kib_per_job": {k: jb["WRITE_SIZE"].get(k, 0.0) / n_jobs for k in keys},
               "rule": "per job: 2 x FETCH_SIZE + WRITE_SIZE (KiB) summed over the stage's kernels; job = every "
                       "dispatch from the first k_map on (fills, copies and scans included)"}
        json.dump(doc, open(a.stages_out, "w"), indent=1)
        print("stages", json.dumps(doc))
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
