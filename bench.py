#!/usr/bin/env python3
"""Benchmark: word-count input GB/s (whole node) on MI355X + % of the HBM roofline.

BASELINE.json metric: "word-count input GB/s (whole node) at 1/2/4/8 MI355X + % of HBM roofline".
Workload (N = 1): configs[2] = C3, wc on 10 GiB of synthetic Zipf(1.1) ASCII text (40 files x 256 MiB,
vocabulary 2^20, nReduce = 64), generated in HBM.  N > 1: C4's shape, 50 files (12.5 GiB) per GPU
(400 files = 100 GiB at N = 8), nReduce = 64, owner(r) = r % N, the shuffle = libmrgpu.so's own RCCL
exchange over xGMI (mrg_job_shuffle; torch.distributed only hands out the communicator id).
Weak scaling: per-GPU work is fixed.  --workload unique: configs[4] (C5), near-unique 12-char keys.

A step = one whole job over the resident input: map (tokenize + combine) -> aggregate + SipHash
partition -> [shuffle] -> sort -> format; the output bytes of every mr-{r}.txt are in HBM at the end
of the step.  Input is resident in HBM before the timed region (host I/O and H2D are excluded; the
D2H of the output is measured after the timed loop and reported beside `value`).

`value` = input bytes of all ranks per step / the MEDIAN step time (each step's time is the max over
ranks); `ms_per_step` is that median; the mean over the bracketed K steps is reported as well.

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 via torch.distributed.run.
"""
import argparse
import gzip
import json
import os
import statistics
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
    ap.add_argument("--cpu-slice-mib", type=int, default=1024, help="C3 slice for the W = cores CPU run")
    ap.add_argument("--cpu-w1-mib", type=int, default=128, help="C3 slice for the W = 1 CPU run")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end leg (files on disk -> mrg_run_job)")
    ap.add_argument("--lds-cap", type=int, default=0)
    ap.add_argument("--shuffle-1", action="store_true",
                    help="N = 1 only: run the library's RCCL shuffle in a one-rank communicator every step (the "
                         "C4 export / exchange / import path without peers; a rehearsal, not the C3 metric)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl = the library's RCCL exchange over xGMI (the product); gloo = host-staged exchange "
                         "through torch.distributed, for rehearsing N > 1 with several ranks on one GPU")
    return ap.parse_args()


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def cpu_cores():
    """Host cores this process may use: the cgroup CPU quota if there is one (the GPU box gives a
    1-GPU job a 16-core share of a larger machine), else OMP_NUM_THREADS, else the affinity mask."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            return max(1, min(n, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        return max(1, min(n, int(os.environ["OMP_NUM_THREADS"])))
    return n


def cpu_baseline(slice_files, w1_bytes, n_reduce):
    """The reference CPU path, restated (oracle/oracle.c FAITHFUL tasks: whole-file read, one write(2)
    + one log line per token into mr-{m}-{r}.txt, read-back, stable sort, grouping), run by W worker
    threads that pull map task ids and then reduce task ids like W `mrworker` processes
    (src/bin/mrworker.rs:43-149).  BASELINE.md: W = host cores and W = 1, on C1 and a C3 slice."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    W = cpu_cores()
    c1 = [gzip.open(os.path.join(ROOT, "tests", "golden", "corpus", f"gut-{m}.txt.gz")).read() for m in range(6)]
    runs = []

    def run(files, R, w, what):
        n = sum(len(f) for f in files)
        with tempfile.TemporaryDirectory(prefix="mr_cpu_") as d:
            t0 = time.perf_counter()
            O.wc_workers(files, R, w, workdir=d)
            dt = time.perf_counter() - t0
        runs.append({"input": what, "bytes": n, "workers": w, "s": round(dt, 3), "GB/s": round(n / dt / 1e9, 6)})
        log(f"cpu baseline: {what}, W={w}: {dt:.2f} s = {n / dt / 1e6:.1f} MB/s")
        return n / dt / 1e9

    run(c1, 10, 1, "C1 bundled corpus (6 files, nReduce 10)")
    run(c1, 10, W, "C1 bundled corpus (6 files, nReduce 10)")
    joined = b"".join(slice_files)
    w1 = [joined[:w1_bytes]]
    run(w1, n_reduce, 1, f"first {w1_bytes // MIB} MiB of the C3 input as one file, nReduce {n_reduce}")
    v = run(slice_files, n_reduce, W, f"first {len(joined) // MIB} MiB of the C3 input as {len(slice_files)} files, "
                                      f"nReduce {n_reduce}")
    return {"value": round(v, 6), "unit": "GB/s", "cores": W, "kind": "port",
            "sample": f"first {len(joined) // MIB} MiB of the benchmark's own C3 input cut into {len(slice_files)} "
                      f"map tasks, nReduce {n_reduce}, W = {W} worker threads (the host cores given to this job) "
                      f"running the reference's task structure (oracle/oracle.c restatement; no Rust toolchain)",
            "runs": runs}


def end_to_end(buf, files, fbytes, n_reduce):
    """SURVEY §8(d) end-to-end leg: the benchmark's own input written to local disk as data/gut-{m}.txt
    files, then the whole job through mrg_run_job (the reference's read -> map -> reduce -> mr-{r}.txt
    path, worker.rs:65-77, 167-179): file reads through pinned staging overlapped with the H2D copies,
    the job, the D2H of the output and the mr-{r}.txt writes.  The files were just written, so they are
    read from the page cache.  Also the C1 latency (the bundled 6-file corpus, nReduce 10)."""
    d = tempfile.mkdtemp(prefix="mrg_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        paths = []
        host = torch.empty(fbytes, dtype=torch.uint8, pin_memory=True)
        for i in range(files):
            host.copy_(buf[i * fbytes:(i + 1) * fbytes])
            pth = os.path.join(d, f"gut-{i}.txt")
            with open(pth, "wb") as f:
                f.write(host.numpy().tobytes())
            paths.append(pth)
        del host
        out = os.path.join(d, "out")
        os.makedirs(out)
        runs = []
        for _ in range(2):  # the first run also faults in the library's host-side setup
            t0 = time.perf_counter()
            st = M.native.run_job(paths, n_reduce, M.APP_WC, out)
            runs.append((time.perf_counter() - t0, st))
        wall, st = min(runs, key=lambda x: x[0])
        n = files * fbytes
        c1 = [gzip.open(os.path.join(ROOT, "tests", "golden", "corpus", f"gut-{m}.txt.gz")).read() for m in range(6)]
        c1p = []
        for m, b in enumerate(c1):
            pth = os.path.join(d, f"c1-{m}.txt")
            with open(pth, "wb") as f:
                f.write(b)
            c1p.append(pth)
        lat = []
        for _ in range(5):
            t0 = time.perf_counter()
            M.native.run_job(c1p, 10, M.APP_WC, out)
            lat.append((time.perf_counter() - t0) * 1e3)
        res = {"end_to_end_gbs": round(n / wall / 1e9, 3), "ms": round(wall * 1e3, 1),
               "phases_ms": {k: round(st[k], 1) for k in ("ms_open", "ms_read", "ms_map", "ms_shuffle", "ms_reduce",
                                                          "ms_write")},
               "input_bytes": n, "output_bytes": st["output_bytes"],
               "read_gbs": round(n / (st["ms_read"] / 1e3) / 1e9, 2) if st["ms_read"] > 0 else None,
               "c1_latency_ms": round(statistics.median(lat), 2),
               "note": "mrg_run_job over the C3 input as %d files on local disk (page cache: written just before), "
                       "nReduce %d: open + read/H2D + map + reduce + D2H + mr-{r}.txt writes; best of 2 runs; "
                       "C1 = bundled corpus, median of 5" % (files, n_reduce)}
        log(f"end-to-end: {res['end_to_end_gbs']} GB/s ({res['ms']} ms: {res['phases_ms']}), C1 {res['c1_latency_ms']} ms")
        return res
    finally:
        import shutil
        shutil.rmtree(d, ignore_errors=True)


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
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    comm = S.library_comm(ctx) if (world > 1 and a.backend == "nccl") else None
    if world == 1 and a.shuffle_1:
        comm = M.Comm(ctx, M.comm_id(), 1, 0)
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
        if comm is not None:
            ctx.shuffle(comm)             # RCCL inside libmrgpu.so, owner(r) = r % N
        elif world > 1:
            S.shuffle(ctx, world, dev)    # host-staged rehearsal (gloo)
        return ctx.reduce()               # ends with a host read of the output size

    for w in range(a.warmup):
        t_w = time.perf_counter()
        step()
        if rank == 0:
            log(f"warmup {w + 1}/{a.warmup}: {time.perf_counter() - t_w:.3f} s  {ctx.stats()}")
    # kernel time of the dominant kernel: HIP events on the library's stream (= torch's current
    # stream, set above) around every k_map launch
    ctx.set_timing(True)
    stats = []
    step_s = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    out_bytes = 0
    for _ in range(a.steps):
        ts = time.perf_counter()
        out_bytes = step()
        step_s.append(time.perf_counter() - ts)
        s = ctx.stats()
        stats.append(s)
        if rank == 0:
            log(f"step: map {s['ms_map']:.2f} ms ({s['map_launches']} launch), agg {s['ms_aggregate']:.2f}, "
                f"sort {s['ms_sort']:.2f}, format {s['ms_format']:.2f}"
                + (f", exchange {s['ms_exchange']:.2f}" if comm is not None or world > 1 else "")
                + f"; wall {step_s[-1] * 1e3:.2f}")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ctx.set_timing(False)
    t = torch.tensor([dt] + step_s, dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt, step_max = t[0].item(), t[1:].tolist()
    med = statistics.median(step_max)
    st = ctx.stats()

    # D2H of the mr-{r}.txt bytes into a pinned host buffer (what a worker writing the files pays
    # over PCIe; not in `value`: reported beside it).  The buffer is allocated outside the timing.
    _, out_off = ctx.output()
    out_n = out_off[-1]
    host_out = torch.empty(max(out_n, 1), dtype=torch.uint8, pin_memory=True)
    host_out.zero_()  # first touch of the pages outside the timing (a 15 GB C5 output otherwise faults them in)
    torch.cuda.synchronize(dev)
    td = time.perf_counter()
    ctx.copy_output_to(host_out.data_ptr(), out_n)
    d2h_ms = (time.perf_counter() - td) * 1e3
    del host_out

    value = shard * world / med / 1e9
    map_ms = [s["ms_map"] for s in stats]
    med_map_ms = statistics.median(map_ms)
    achieved = shard / (med_map_ms / 1e3) / 1e9  # algorithmic bytes per k_map launch = input bytes read once
    traffic, traffic_note = None, "no PMC measurement for this kernel source"
    tpath = os.path.join(ROOT, "profiles", "map_traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if tj.get("kernel_src_sha") != M.native.kernel_source_sha():
            traffic_note = "profiles/map_traffic.json was measured on other kernel sources: not reported"
        elif tj.get("input_bytes") != shard:
            traffic_note = "profiles/map_traffic.json was measured on another input size: not reported"
        else:
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_note = ("rocprofv3 PMC of this kernel source (kernel_src_sha %s): 2 x FETCH_SIZE + WRITE_SIZE "
                            "per k_map launch, profiles/map_traffic.json" % tj["kernel_src_sha"])

    # xGMI roofline of the exchange (N > 1 over RCCL): peer bytes per rank (max of sent and received)
    # / the HIP-event time of the send/recv group, against (N - 1) links x 153 GB/s one way (each GPU
    # of the node has a direct link to each peer).  Max over ranks of time and bytes.
    xgmi = None
    if comm is not None and world > 1:
        ex_ms = statistics.median(s["ms_exchange"] for s in stats)
        ex_b = max(statistics.median(s["exchange_sent"] for s in stats),
                   statistics.median(s["exchange_recv"] for s in stats))
        tx = torch.tensor([ex_ms, ex_b], dtype=torch.float64, device=dev)
        dist.all_reduce(tx, op=dist.ReduceOp.MAX)
        ex_ms, ex_b = tx.tolist()
        peak = (world - 1) * XGMI_LINK_GBS
        ach = ex_b / (ex_ms / 1e3) / 1e9 if ex_ms > 0 else 0.0
        xgmi = {"bytes_per_rank": int(ex_b), "ms_exchange": round(ex_ms, 3), "achieved": round(ach, 1),
                "peak": peak, "unit": "GB/s", "frac": round(ach / peak, 4),
                "note": "libmrgpu RCCL send/recv group: max-over-ranks peer bytes / HIP-event time (median step)"}

    wl = {"zipf": ("C3: wc, Zipf(%.2f) ASCII text, vocab %d" % (a.zipf_s, a.vocab)) if world == 1 else
          ("C4: wc, Zipf(%.2f) text sharded over %d GPUs, %s shuffle"
           % (a.zipf_s, world, "RCCL" if a.backend == "nccl" else "gloo (host-staged rehearsal)")),
          "unique": "C5: near-unique 12-char keys (1% repeats)" + ("" if world == 1 else ", %d GPUs" % world)}
    line = {
        "metric": "word-count input GB/s (whole node) at 1/2/4/8 MI355X + % of HBM roofline",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(med * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": wl[a.workload] + (" + one-rank RCCL shuffle rehearsal" if a.shuffle_1 and world == 1 else ""), "input_bytes_per_gpu": shard, "files_per_gpu": files,
                   "file_bytes": fbytes, "n_reduce": a.reduce, "parallelism": f"shard{world}"},
        "roofline": {"bound": "hbm", "kernel": "k_map (tokenize + LDS combine)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_note": traffic_note,
                     "algorithmic_bytes_per_launch": shard, "kernel_ms_median": round(med_map_ms, 3),
                     "whole_job_frac": round(value / world / HBM_PEAK_GBS, 4)},
        "xgmi": xgmi,
        "timing": {"value_basis": "median step (max over ranks)", "ms_per_step_mean": round(dt / a.steps * 1e3, 3),
                   "value_mean": round(shard * world * a.steps / dt / 1e9, 3),
                   "output_d2h_ms": round(d2h_ms, 3),
                   "value_with_output_d2h": round(shard * world / (med + d2h_ms / 1e3) / 1e9, 3)},
        "stages_ms": {k: round(statistics.median(s[k] for s in stats), 3)
                      for k in ("ms_map", "ms_aggregate", "ms_sort", "ms_format")},
        "job": {"tokens": st["tokens"], "map_records": st["map_records"], "distinct_keys": st["distinct_keys"],
                "output_bytes": out_bytes, "map_launches": [s["map_launches"] for s in stats]},
    }
    if world == 1 and not a.no_e2e and a.workload == "zipf":
        line["end_to_end"] = end_to_end(buf, files, fbytes, a.reduce)
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.workload == "zipf":
        n = min(a.cpu_slice_mib * MIB, shard)
        host = buf[:n].cpu().numpy().tobytes()
        W = cpu_cores()
        per = n // W
        # cut at a space so each map task holds whole tokens (the C3 generator separates words by ' ')
        cuts = [0]
        for i in range(1, W):
            j = host.find(b" ", i * per)
            cuts.append(j if j > 0 else cuts[-1])
        cuts.append(n)
        slice_files = [host[cuts[i]:cuts[i + 1]] for i in range(W)]
        line["cpu_baseline"] = cpu_baseline(slice_files, min(a.cpu_w1_mib * MIB, n), a.reduce)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
