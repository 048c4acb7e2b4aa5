#!/usr/bin/env python3
"""Benchmark: word-count input GB/s (whole node) on MI355X + % of the HBM roofline.

BASELINE.json metric: "word-count input GB/s (whole node) at 1/2/4/8 MI355X + % of HBM roofline".
Workload (N = 1): configs[2] = C3, wc on 10 GiB of synthetic Zipf(1.1) ASCII text (40 files x 256 MiB,
vocabulary 2^20, nReduce = 64), generated in HBM.  N > 1: C4's shape, 50 files (12.5 GiB) per GPU
(400 files = 100 GiB at N = 8), nReduce = 64, shuffle = all-to-all over RCCL (torch.distributed
"nccl"), owner(r) = r % N.  Weak scaling: per-GPU work is fixed.

A step = one whole job over the resident input: map (tokenize + combine) -> aggregate + SipHash
partition -> [export -> all-to-all -> import] -> sort -> format; the output bytes of every
mr-{r}.txt are in HBM at the end of the step.  Input is resident in HBM before the timed region
(host I/O and H2D are excluded; see DESIGN.md for the end-to-end numbers).

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 via torch.distributed.run.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import mapreduce_rust_amd as M  # noqa: E402
from mapreduce_rust_amd import shuffle as S  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
XGMI_LINK_GBS = 153.0  # one xGMI link, one direction; 7 links per GPU, one to each peer of the node
MIB = 1 << 20


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["zipf", "unique"], default="zipf")
    ap.add_argument("--files-per-gpu", type=int, default=0, help="0: 40 at N=1 (C3), 50 at N>1 (C4)")
    ap.add_argument("--file-mib", type=int, default=256)
    ap.add_argument("--reduce", type=int, default=64)
    ap.add_argument("--vocab", type=int, default=1 << 20)
    ap.add_argument("--zipf-s", type=float, default=1.1)
    ap.add_argument("--seed", type=int, default=0x5EED2026)
    ap.add_argument("--cpu-sample-mib", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lds-cap", type=int, default=0)
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = RCCL over xGMI (the product); gloo = host-staged exchange, for rehearsing N > 1 "
                         "with several ranks on one GPU")
    return ap.parse_args()


def cpu_baseline(sample, n_reduce):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    res = {}
    with tempfile.TemporaryDirectory(prefix="mr_cpu_") as d:
        t0 = time.perf_counter()
        O.wc([sample], n_reduce, O.FAITHFUL, workdir=d)
        res["faithful_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    O.wc([sample], n_reduce, O.FAST)
    res["fast_s"] = time.perf_counter() - t0
    return res


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    gpu = local % max(1, torch.cuda.device_count())  # = local on a node with one GPU per rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    files = a.files_per_gpu or (40 if world == 1 else 50)
    fbytes = a.file_mib * MIB
    shard = files * fbytes

    if a.lds_cap:
        os.environ["MRG_LDS_CAP"] = str(a.lds_cap)
    ctx = M.Context(gpu)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    buf = torch.empty(shard + 64, dtype=torch.uint8, device=dev)
    for i in range(files):
        fi = rank * files + i
        p = buf.data_ptr() + i * fbytes
        if a.workload == "zipf":
            ctx.gen_zipf(p, fbytes, a.seed, fi, a.vocab, a.zipf_s)
        else:
            ctx.gen_unique(p, fbytes, a.seed, fi)
        if rank == 0 and (i % 8 == 7 or i == files - 1):
            torch.cuda.synchronize(dev)
            log(f"generated {i + 1}/{files} files of {a.file_mib} MiB")
    torch.cuda.synchronize(dev)
    doc_off = [i * fbytes for i in range(files + 1)]
    doc_ids = [rank * files + i for i in range(files)]

    def step():
        ctx.job_begin(M.APP_WC, a.reduce)
        ctx.set_input(buf.data_ptr(), doc_off, doc_ids)
        ctx.map()
        if world > 1:
            S.shuffle(ctx, world, dev)  # RCCL all-to-all over xGMI, owner(r) = r % N
        return ctx.reduce()

    for w in range(a.warmup):
        t_w = time.perf_counter()
        step()
        if rank == 0:
            log(f"warmup {w + 1}/{a.warmup}: {time.perf_counter() - t_w:.3f} s  {ctx.stats()}")
    ctx.set_timing(True)
    map_ms = []
    stage = {"ms_map": 0.0, "ms_aggregate": 0.0, "ms_sort": 0.0, "ms_format": 0.0}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    S.EXCHANGES.clear()
    t0 = time.perf_counter()
    out_bytes = 0
    t_prev = t0
    for _ in range(a.steps):
        out_bytes = step()
        t_now = time.perf_counter()
        wall_ms = (t_now - t_prev) * 1e3  # the step ends with a host read of the output size
        t_prev = t_now
        s = ctx.stats()
        map_ms.append(s["ms_map"])
        for k in stage:
            stage[k] += s[k] / a.steps
        if rank == 0:
            log(f"step: map {s['ms_map']:.2f} ms ({s['map_launches']} launch), agg {s['ms_aggregate']:.2f}, "
                f"sort {s['ms_sort']:.2f}, format {s['ms_format']:.2f}; wall {wall_ms:.2f}")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    st = ctx.stats()

    total_in = shard * world * a.steps
    value = total_in / dt / 1e9
    avg_map_ms = sum(map_ms) / len(map_ms)
    achieved = shard / (avg_map_ms / 1e3) / 1e9  # algorithmic bytes per launch = input bytes read
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "map_traffic.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("input_bytes") == shard:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # xGMI roofline of the exchange (N > 1 over RCCL): peer bytes per rank (max of sent and received)
    # / average time of the data all-to-alls, against (N - 1) links x 153 GB/s one way (each GPU of
    # the node has a direct link to each peer).  Max over ranks of the time, sum of the bytes.
    xgmi = None
    if world > 1 and S.EXCHANGES:
        ex_ms = sum(e["start"].elapsed_time(e["end"]) for e in S.EXCHANGES) / len(S.EXCHANGES)
        ex_b = max(sum(e["sent"] for e in S.EXCHANGES), sum(e["received"] for e in S.EXCHANGES)) / len(S.EXCHANGES)
        tx = torch.tensor([ex_ms, ex_b], dtype=torch.float64, device=dev)
        dist.all_reduce(tx, op=dist.ReduceOp.MAX)
        ex_ms, ex_b = tx.tolist()
        peak = (world - 1) * XGMI_LINK_GBS
        ach = ex_b / (ex_ms / 1e3) / 1e9 if ex_ms > 0 else 0.0
        xgmi = {"bytes_per_rank": int(ex_b), "ms_exchange": round(ex_ms, 3), "achieved": round(ach, 1),
                "peak": peak, "unit": "GB/s", "frac": round(ach / peak, 4),
                "note": "max-over-ranks peer bytes of the record + heap all-to-alls / their event time"}

    line = {
        "metric": "word-count input GB/s (whole node) at 1/2/4/8 MI355X + % of HBM roofline",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(dt / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": ("C3: wc, Zipf(%.2f) ASCII text, vocab %d" % (a.zipf_s, a.vocab))
                   if (a.workload == "zipf" and world == 1) else
                   ("C4: wc, Zipf(%.2f) text sharded over %d GPUs, RCCL all-to-all" % (a.zipf_s, world)
                    if a.workload == "zipf" else "C5: near-unique 12-char keys"),
                   "input_bytes_per_gpu": shard, "files_per_gpu": files, "file_bytes": fbytes,
                   "n_reduce": a.reduce, "parallelism": f"shard{world}"},
        "roofline": {"bound": "hbm", "kernel": "k_map (tokenize + LDS combine)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "whole_job_frac": round(value / world / HBM_PEAK_GBS, 4)},
        "xgmi": xgmi,
        "stages_ms": {k: round(v, 3) for k, v in stage.items()},
        "job": {"tokens": st["tokens"], "map_records": st["map_records"], "distinct_keys": st["distinct_keys"],
                "output_bytes": out_bytes},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        n = min(a.cpu_sample_mib * MIB, shard)
        sample = buf[:n].cpu().numpy().tobytes()
        log(f"cpu baseline on {n // MIB} MiB ...")
        cb = cpu_baseline(sample, a.reduce)
        line["cpu_baseline"] = {"value": round(n / cb["faithful_s"] / 1e9, 6), "unit": "GB/s", "cores": 1,
                                "kind": "port",
                                "sample": f"first {n // MIB} MiB of the same input, reference structure (per-token "
                                          f"write(2) + log line, intermediate files, stable sort), 1 thread",
                                "fast_inmemory_value": round(n / cb["fast_s"] / 1e9, 6)}
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
