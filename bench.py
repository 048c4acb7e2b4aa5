#!/usr/bin/env python3
"""Benchmark: word-count input GB/s (whole node) on MI355X + % of the HBM roofline.

BASELINE.json metric: "word-count input GB/s (whole node) at 1/2/4/8 MI355X + % of HBM roofline".
Workload (N = 1): configs[2] = C3, wc on 10 GiB of synthetic Zipf(1.1) ASCII text (40 files x 256 MiB,
vocabulary 2^20, nReduce = 64), generated in HBM.  N > 1: C4's shape, 50 files (12.5 GiB) per GPU
(400 files = 100 GiB at N = 8), nReduce = 64, owner(r) = r % N, the shuffle = libmrgpu.so's own RCCL
exchange over xGMI (mrg_job_shuffle; torch.distributed only hands out the communicator id).
Weak scaling: per-GPU work is fixed.  --workload unique: configs[4] (C5), near-unique 12-char keys;
--workload zipf_u: the C3 text with Gutenberg-like Unicode (the reference corpus's kind of text).

The default N = 1 run adds, beside the C3 line: a `cold` object (the first job on a fresh Context over
the same resident input -- what mrg_run_job and every one-shot worker call run -- with the pool's device
allocations reported apart from the kernels), the end-to-end leg (files on disk -> mrg_run_job), a
zipf_u sub-object (k_map GB/s on Unicode text against the ASCII rate), a c5 sub-object (configs[4] at
50 x 256 MiB, 3 timed steps, with its own `cold` object), a c2 sub-object (the indexer's latency on the
bundled corpus, configs[1]) and the CPU baseline; --quick leaves all of them out.

A step = one whole job over the resident input: map (tokenize + combine) -> aggregate + SipHash
partition -> [shuffle] -> sort -> format; the output bytes of every mr-{r}.txt are in HBM at the end
of the step.  Input is resident in HBM before the timed region (host I/O and H2D are excluded; the
D2H of the output is measured after the timed loop and reported beside `value`).

`value` = input bytes of all ranks per step / the MEDIAN step time (each step's time is the max over
ranks); `ms_per_step` is that median; the mean over the bracketed K steps is reported as well.

Launch: python bench.py [--gpus N --steps K --warmup W].  N > 1: under torch.distributed.run (one rank
per GPU), or without a launcher, when bench.py starts the N ranks itself before touching the GPU; it
exits non-zero if fewer than N GPUs are visible, and the line carries `rccl_nranks` (ncclCommCount of
the library's communicator) beside `n_gpus`.
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
    ap.add_argument("--workload", choices=["zipf", "zipf_u", "unique"], default="zipf",
                    help="zipf: C3 ASCII; zipf_u: the same Zipf text with Gutenberg-like Unicode; unique: C5")
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
    ap.add_argument("--no-zipf-u", action="store_true", help="skip the Gutenberg-like Unicode leg (N = 1)")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 leg (N = 1)")
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 indexer latency leg (N = 1)")
    ap.add_argument("--quick", action="store_true", help="the headline C3 line only (no extra legs)")
    ap.add_argument("--c5-files", type=int, default=50, help="C5 leg: 256 MiB files (50 = configs[4]'s 1e9 keys)")
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
               "phases_ms": {k: round(st[k], 2) for k in ("ms_open", "ms_read", "ms_map", "ms_map_alloc", "ms_map_kernel",
                                                          "ms_aggregate_kernel", "ms_shuffle", "ms_reduce", "ms_write")},
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


WL_LABEL = {"zipf": "C3: wc, Zipf(%.2f) ASCII text, vocab %d",
            "zipf_u": "C3 text with Gutenberg-like Unicode (U+2019/201C/201D/2014, U+00E9): wc, Zipf(%.2f), vocab %d",
            "unique": "C5: near-unique 12-char keys (1% repeats)"}


def generate(ctx, buf, workload, files, fbytes, rank, a, dev, quiet=False):
    for i in range(files):
        fi = rank * files + i
        p = buf.data_ptr() + i * fbytes
        if workload == "zipf":
            ctx.gen_zipf(p, fbytes, a.seed, fi, a.vocab, a.zipf_s)
        elif workload == "zipf_u":
            ctx.gen_text(p, fbytes, a.seed, fi, a.vocab, a.zipf_s, 1)
        else:
            ctx.gen_unique(p, fbytes, a.seed, fi)
        if rank == 0 and not quiet and (i % 8 == 7 or i == files - 1):
            torch.cuda.synchronize(dev)
            log(f"generated {i + 1}/{files} {workload} files of {fbytes // MIB} MiB")
    torch.cuda.synchronize(dev)


def time_steps(ctx, step, steps, warmup, dev, world, rank, label):
    """W untimed warmup steps, then K steps bracketed by a barrier + synchronize on both sides; per-step
    wall times (max over ranks) and the library's per-stage stats of every timed step."""
    for w in range(warmup):
        t_w = time.perf_counter()
        step()
        if rank == 0:
            log(f"{label} warmup {w + 1}/{warmup}: {time.perf_counter() - t_w:.3f} s  {ctx.stats()}")
    # kernel time of every stage: HIP events on the library's stream (= torch's current stream)
    ctx.set_timing(True)
    stats, step_s = [], []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        ts = time.perf_counter()
        step()
        step_s.append(time.perf_counter() - ts)
        s = ctx.stats()
        stats.append(s)
        if rank == 0:
            log(f"{label} step: map {s['ms_map']:.2f} ms ({s['map_launches']} launch), agg {s['ms_aggregate']:.2f}, "
                f"sort {s['ms_sort']:.2f}, format {s['ms_format']:.2f}"
                + (f", exchange {s['ms_exchange']:.2f}" if world > 1 else "")
                + f"; wall {step_s[-1] * 1e3:.2f}")
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ctx.set_timing(False)
    t = torch.tensor([dt] + step_s, dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t[0].item(), t[1:].tolist(), stats


def med(stats, k):
    return statistics.median(s[k] for s in stats)


def stage_roofline(stats, shard, out_bytes):
    """Per-stage roofline: median HIP-event ms of each stage, its
    algorithmic bytes per job, achieved GB/s and fraction of HBM peak; PMC bytes per job from
    profiles/stage_traffic.json when it was measured on these kernel sources and this input size."""
    st = stats[-1]
    keys, tail, t16 = st["distinct_keys"], st["map_records"], st["tail_records_16"]
    rec_bytes = 12 * (tail - t16) + 16 * t16
    algo = {
        "map": (shard, "input bytes, read once"),
        "aggregate": (rec_bytes + 36 * keys, "tail records read (12 or 16 B each) + 36 B per distinct key written"),
        "sort": (5 * 32 * keys, "a 32-B sort record per key: written, read + written by the scatter, by the leaf sort"),
        "format": (out_bytes + 2 * 32 * keys, "output bytes written + the sort records read twice (lengths, write)"),
    }
    ms_key = {"map": "ms_map", "aggregate": "ms_aggregate", "sort": "ms_sort", "format": "ms_format"}
    pmc, note = None, "no PMC measurement for these kernel sources"
    tpath = os.path.join(ROOT, "profiles", "stage_traffic.json")
    if os.path.exists(tpath):
        tj = json.load(open(tpath))
        if tj.get("kernel_src_sha") != M.native.kernel_source_sha():
            note = "profiles/stage_traffic.json was measured on other kernel sources: not reported"
        elif tj.get("input_bytes") != shard:
            note = "profiles/stage_traffic.json was measured on another input size: not reported"
        else:
            pmc = tj
            note = ("rocprofv3 PMC of these kernel sources (kernel_src_sha %s): per job, 2 x FETCH_SIZE + WRITE_SIZE "
                    "over the stage's kernels, profiles/stage_traffic.json" % tj["kernel_src_sha"])
    stages = {}
    for k, (b, what) in algo.items():
        ms = med(stats, ms_key[k])
        ach = b / (ms / 1e3) / 1e9 if ms > 0 else None
        stages[k] = {"ms_median": round(ms, 3), "algorithmic_bytes": int(b), "algorithmic": what,
                     "achieved_gbs": round(ach, 1) if ach else None,
                     "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                     "pmc_bytes": pmc["stage_hbm_bytes"].get(k) if pmc else None,
                     "pmc_gbs": round(pmc["stage_hbm_bytes"][k] / (ms / 1e3) / 1e9, 1) if pmc and ms > 0 else None}
    ratio = round(pmc["job_hbm_bytes"] / shard, 3) if pmc else None
    return stages, ratio, note


def cold_job(dev, buf, doc_off, n_reduce, steady, cached=False):
    """The FIRST job on a fresh Context over the same resident input: what mrg_run_job and every
    one-shot worker call run (the reference runs each task once per call, src/bin/mrworker.rs:95,145).
    Reports its wall time, its kernel time (sum of the HIP-event stages) against the steady steps'
    median, the pool's device allocations (hipMalloc calls, bytes, host ms: paid once per context, so
    reported apart from the kernels) and the paths it took.  `steady` = the warm legs' per-step stats."""
    ctx = M.Context(dev.index)
    try:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        ctx.set_timing(True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ctx.job_begin(M.APP_WC, n_reduce)
        ctx.set_input(buf.data_ptr(), doc_off)
        ctx.map()
        ctx.reduce()
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t0) * 1e3
        st = ctx.stats()
        n_alloc, alloc_bytes, alloc_ms = ctx.pool_alloc_stats()
    finally:
        ctx.close()
    keys = ("ms_map", "ms_aggregate", "ms_sort", "ms_format")
    kern = sum(st[k] for k in keys)
    warm = statistics.median(sum(s[k] for k in keys) for s in steady)
    res = {"ms_wall": round(wall, 3), "ms_kernels": round(kern, 3), "steady_ms_kernels": round(warm, 3),
           "kernels_vs_steady": round(kern / warm, 3) if warm > 0 else None,
           "stages_ms": {k: round(st[k], 3) for k in keys},
           "pool_allocs": n_alloc, "pool_alloc_bytes": alloc_bytes, "pool_alloc_ms": round(alloc_ms, 3),
           "ms_wall_minus_alloc": round(wall - alloc_ms, 3),
           "map_launches": st["map_launches"], "map_kind": st["map_kind"], "agg_path": st["agg_path"],
           "blocks": "from the device cache (the warm leg's Context closed first)" if cached else
                     "fresh device memory (the warm Context still open)",
           "note": "first job on a fresh Context (same resident input, same process): wall = job_begin .. reduce; "
                   "kernels = sum of the HIP-event stages; pool_alloc_ms = host time inside the pool's hipMalloc calls"}
    log(f"cold job: wall {res['ms_wall']} ms (alloc {res['pool_alloc_ms']} ms in {n_alloc} hipMalloc), kernels "
        f"{res['ms_kernels']} ms vs steady {res['steady_ms_kernels']}, map launches {res['map_launches']}, "
        f"map kind {res['map_kind']}")
    return res


def leg(dev, a, workload, files, steps, warmup):
    """An extra single-GPU workload (zipf_u, C5) on its own buffer and its own Context, timed like the
    headline line.  The Context is closed after the timed steps, so its device blocks go to the
    library's per-device cache (as a worker's do between mrg_run_job calls); C5's cold job then opens
    a fresh Context over them -- beside a live warm context the two held ~130 GB of the 288, and a
    device-full trim frees memory the driver must wipe before reuse (seconds: DESIGN.md section 15.4)."""
    fbytes = a.file_mib * MIB
    shard = files * fbytes
    buf = torch.empty(shard + 64, dtype=torch.uint8, device=dev)
    ctx = M.Context(dev.index)
    try:
        ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        generate(ctx, buf, workload, files, fbytes, 0, a, dev, quiet=True)
        doc_off = [i * fbytes for i in range(files + 1)]

        def step():
            ctx.job_begin(M.APP_WC, a.reduce)
            ctx.set_input(buf.data_ptr(), doc_off)
            ctx.map()
            return ctx.reduce()

        dt, step_max, stats = time_steps(ctx, step, steps, warmup, dev, 1, 0, workload)
    finally:
        ctx.close()
    cold = cold_job(dev, buf, doc_off, a.reduce, stats, cached=True) if workload == "unique" else None
    del buf
    torch.cuda.empty_cache()
    m = statistics.median(step_max)
    map_ms = med(stats, "ms_map")
    st = stats[-1]
    tiles = -(-shard // 1024)
    return {"workload": WL_LABEL[workload] if workload == "unique" else WL_LABEL[workload] % (a.zipf_s, a.vocab),
            "input_bytes": shard, "files": files, "n_reduce": a.reduce, "steps": steps, "warmup": warmup,
            "value": round(shard / m / 1e9, 3), "unit": "GB/s", "ms_per_step": round(m * 1e3, 3),
            "k_map_ms_median": round(map_ms, 3), "k_map_gbs": round(shard / (map_ms / 1e3) / 1e9, 1),
            "stages_ms": {k: round(med(stats, k), 3) for k in ("ms_map", "ms_aggregate", "ms_sort", "ms_format")},
            "tokens": st["tokens"], "long_tokens": st["long_tokens"], "map_records": st["map_records"],
            "distinct_keys": st["distinct_keys"], "nonascii_tiles": st["nonascii_tiles"],
            "nonascii_tile_frac": round(st["nonascii_tiles"] / tiles, 4), "agg_path": st["agg_path"],
            **({"cold": cold} if cold else {})}


def c2_latency(ctx, dev):
    """configs[1]: the indexer (word -> sorted unique documents) on the bundled corpus, nReduce 10:
    latency of the whole job with the corpus resident in HBM (median of 5, after one warmup) and
    through mrg_run_job from files on disk (read + H2D + job + D2H + mr-{r}.txt writes)."""
    c1 = [gzip.open(os.path.join(ROOT, "tests", "golden", "corpus", f"gut-{m}.txt.gz")).read() for m in range(6)]
    names = [f"data/gut-{m}.txt" for m in range(6)]
    off = [0]
    for b in c1:
        off.append(off[-1] + len(b))
    buf = torch.frombuffer(bytearray(b"".join(c1) + bytes(64)), dtype=torch.uint8).to(dev)
    lat = []
    ctx.set_timing(True)
    for i in range(6):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ctx.job_begin(M.APP_INDEXER, 10)
        ctx.set_doc_names(names)
        ctx.set_input(buf.data_ptr(), off)
        ctx.map()
        n_out = ctx.reduce()
        if i:
            lat.append((time.perf_counter() - t0) * 1e3)
    st = ctx.stats()
    ctx.set_timing(False)
    d = tempfile.mkdtemp(prefix="mrg_c2_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        os.makedirs(os.path.join(d, "data"))
        paths = []
        for m, b in enumerate(c1):
            pth = os.path.join(d, "data", f"gut-{m}.txt")
            with open(pth, "wb") as f:
                f.write(b)
            paths.append(pth)
        e2e = []
        for i in range(6):
            t0 = time.perf_counter()
            M.native.run_job(paths, 10, M.APP_INDEXER, d)
            if i:
                e2e.append((time.perf_counter() - t0) * 1e3)
    finally:
        import shutil
        shutil.rmtree(d, ignore_errors=True)
    res = {"workload": "C2: indexer on the bundled corpus (6 files, 4.1 MB), nReduce 10",
           "latency_ms_resident": round(statistics.median(lat), 3),
           "latency_ms_end_to_end": round(statistics.median(e2e), 3),
           "stages_ms": {k: round(st[k], 3) for k in ("ms_map", "ms_aggregate", "ms_sort", "ms_format")},
           "distinct_keys": st["distinct_keys"], "output_bytes": n_out,
           "note": "resident: job_begin .. reduce (output in HBM), median of 5 after a warmup; end_to_end: "
                   "mrg_run_job over the 6 files on disk incl. the mr-{r}.txt writes, median of 5"}
    log(f"C2 indexer: {res['latency_ms_resident']} ms resident, {res['latency_ms_end_to_end']} ms end to end")
    return res


def launch_plan(gpus, backend, env, n_devices):
    """How this process runs `--gpus N` (decided before anything touches the GPU):
    "single" -- N = 1, no launcher: this process is the only rank;
    "spawn"  -- N > 1, no launcher (WORLD_SIZE unset): start N rank processes through
                torch.distributed.run on this node and exit with their status;
    "rank"   -- started by a launcher as one of WORLD_SIZE ranks.
    Raises SystemExit when N does not match the launcher's WORLD_SIZE, or when the RCCL path would
    put two ranks on one GPU (fewer visible devices than ranks on the node): a multi-GPU bench never
    falls back to measuring fewer GPUs than it reports."""
    world = int(env.get("WORLD_SIZE", "1"))
    if gpus < 1:
        raise SystemExit(f"--gpus {gpus}: need at least 1")
    if world > 1 or ("WORLD_SIZE" in env and gpus > 1):
        if gpus != world:
            raise SystemExit(f"--gpus {gpus} but WORLD_SIZE {world}")
        local_world = int(env.get("LOCAL_WORLD_SIZE", str(world)))
        if backend == "nccl" and n_devices < local_world:
            raise SystemExit(f"{local_world} ranks on this node but only {n_devices} GPU(s) visible: "
                             "the RCCL path needs one GPU per rank")
        return "rank"
    if gpus == 1:
        return "single"
    if backend == "nccl" and n_devices < gpus:
        raise SystemExit(f"--gpus {gpus} but only {n_devices} GPU(s) visible")
    return "spawn"


def spawn_ranks(gpus, argv):
    """N rank processes on this node (torch.distributed.run, rendezvous on 127.0.0.1), started from a
    parent that has not touched the GPU; returns their exit status."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    log(f"--gpus {gpus} without a launcher: starting {gpus} ranks ({' '.join(cmd[1:6])} ...)")
    return subprocess.call(cmd)


def main():
    a = parse()
    plan = launch_plan(a.gpus, a.backend, os.environ, torch.cuda.device_count())
    if plan == "spawn":
        raise SystemExit(spawn_ranks(a.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.quick:
        a.no_e2e = a.no_cpu_baseline = a.no_zipf_u = a.no_c5 = a.no_c2 = True
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
    generate(ctx, buf, a.workload, files, fbytes, rank, a, dev)
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

    dt, step_max, stats = time_steps(ctx, step, a.steps, a.warmup, dev, world, rank, "")
    out_bytes = ctx.stats()["output_bytes"]
    m = statistics.median(step_max)
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

    value = shard * world / m / 1e9
    med_map_ms = med(stats, "ms_map")
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
    stages, job_ratio, stages_note = stage_roofline(stats, shard, out_bytes)

    # xGMI roofline of the exchange (N > 1 over RCCL): peer bytes per rank (max of sent and received)
    # / the HIP-event time of the send/recv group, against (N - 1) links x 153 GB/s one way (each GPU
    # of the node has a direct link to each peer).  Max over ranks of time and bytes.
    xgmi = None
    if comm is not None and world > 1:
        ex_ms = med(stats, "ms_exchange")
        ex_b = max(med(stats, "exchange_sent"), med(stats, "exchange_recv"))
        tx = torch.tensor([ex_ms, ex_b], dtype=torch.float64, device=dev)
        dist.all_reduce(tx, op=dist.ReduceOp.MAX)
        ex_ms, ex_b = tx.tolist()
        peak = (world - 1) * XGMI_LINK_GBS
        ach = ex_b / (ex_ms / 1e3) / 1e9 if ex_ms > 0 else 0.0
        xgmi = {"bytes_per_rank": int(ex_b), "ms_exchange": round(ex_ms, 3), "achieved": round(ach, 1),
                "peak": peak, "unit": "GB/s", "frac": round(ach / peak, 4),
                "note": "libmrgpu RCCL send/recv group: max-over-ranks peer bytes / HIP-event time (median step)"}

    if a.workload == "unique":
        wl = WL_LABEL["unique"] + ("" if world == 1 else ", %d GPUs" % world)
    elif world == 1:
        wl = WL_LABEL[a.workload] % (a.zipf_s, a.vocab)
    else:
        wl = ("C4: wc, Zipf(%.2f) %s text sharded over %d GPUs, %s shuffle"
              % (a.zipf_s, "ASCII" if a.workload == "zipf" else "Gutenberg-like Unicode", world,
                 "RCCL" if a.backend == "nccl" else "gloo (host-staged rehearsal)"))
    # ranks of the library's RCCL communicator as RCCL counts them (ncclCommCount): at N > 1 it must
    # equal n_gpus; null when no communicator exists (N = 1, or the gloo rehearsal)
    rccl_nranks = comm.count() if comm is not None else None
    if world > 1 and a.backend == "nccl" and rccl_nranks != world:
        raise SystemExit(f"RCCL communicator has {rccl_nranks} ranks, WORLD_SIZE is {world}")
    line = {
        "metric": "word-count input GB/s (whole node) at 1/2/4/8 MI355X + % of HBM roofline",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "rccl_nranks": rccl_nranks,
        "devices_visible": torch.cuda.device_count(),
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(m * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": wl + (" + one-rank RCCL shuffle rehearsal" if a.shuffle_1 and world == 1 else ""),
                   "input_bytes_per_gpu": shard, "files_per_gpu": files,
                   "file_bytes": fbytes, "n_reduce": a.reduce, "parallelism": f"shard{world}"},
        "roofline": {"bound": "hbm", "kernel": "k_map (tokenize + LDS combine)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_note": traffic_note,
                     "algorithmic_bytes_per_launch": shard, "kernel_ms_median": round(med_map_ms, 3),
                     "whole_job_frac": round(value / world / HBM_PEAK_GBS, 4),
                     "stages": stages, "whole_job_traffic_ratio": job_ratio, "stages_note": stages_note},
        "xgmi": xgmi,
        "timing": {"value_basis": "median step (max over ranks)", "ms_per_step_mean": round(dt / a.steps * 1e3, 3),
                   "value_mean": round(shard * world * a.steps / dt / 1e9, 3),
                   "output_d2h_ms": round(d2h_ms, 3),
                   "value_with_output_d2h": round(shard * world / (m + d2h_ms / 1e3) / 1e9, 3)},
        "stages_ms": {k: round(med(stats, k), 3) for k in ("ms_map", "ms_aggregate", "ms_sort", "ms_format")},
        "job": {"tokens": st["tokens"], "map_records": st["map_records"], "distinct_keys": st["distinct_keys"],
                "output_bytes": out_bytes, "map_launches": [s["map_launches"] for s in stats],
                "nonascii_tiles": st["nonascii_tiles"], "spec_agg": [s["spec_agg"] for s in stats],
                "agg_path": st["agg_path"]},
    }
    single = world == 1 and a.workload == "zipf" and not a.shuffle_1
    if world == 1 and not a.shuffle_1 and not a.quick:
        line["cold"] = cold_job(dev, buf, doc_off, a.reduce, stats)
    if single and not a.no_e2e:
        line["end_to_end"] = end_to_end(buf, files, fbytes, a.reduce)
    cpu = None
    if rank == 0 and single and not a.no_cpu_baseline:
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
        del host
        cpu = (slice_files, min(a.cpu_w1_mib * MIB, n))
    if single:
        del buf
        torch.cuda.empty_cache()
        if not a.no_zipf_u:
            u = leg(dev, a, "zipf_u", files, 5, 2)
            u["k_map_vs_ascii"] = round(u["k_map_gbs"] / achieved, 4)
            line["zipf_u"] = u
            log(f"zipf_u: {u['value']} GB/s, k_map {u['k_map_gbs']} GB/s = {u['k_map_vs_ascii']} of ASCII, "
                f"{u['nonascii_tile_frac']} of tiles non-ASCII")
        if not a.no_c5:
            c5 = leg(dev, a, "unique", a.c5_files, 3, 1)
            line["c5"] = c5
            log(f"C5: {c5['value']} GB/s ({c5['ms_per_step']} ms per step, {c5['distinct_keys']} keys)")
        if not a.no_c2:
            line["c2"] = c2_latency(ctx, dev)
    if cpu is not None:
        line["cpu_baseline"] = cpu_baseline(cpu[0], cpu[1], a.reduce)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
