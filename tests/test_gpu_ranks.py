"""Multi-rank exchange at C4 / C5 shape, failure paths of the multi-GPU plan, exchange-record edge cases.

* BASELINE configs[3] (C4: Zipf text sharded over GPUs, nReduce 64) and configs[4] (C5: near-unique
  keys) through the library's export -> all-to-all -> import at world 2 and 3, several processes on the
  one GPU (gloo moves the records: RCCL puts one rank per device).  Each rank generates its own files
  (distinct file indices), maps, exchanges, re-aggregates and reduces the partitions it owns; the union
  of the owned mr-{r}.txt equals the oracle's run over all ranks' bytes.  The reference hands the
  partitions over through mr-{m}-{r}.txt files: src/mr/worker.rs:117-140 -> 79-109.
* A rank whose export fails: every rank of the exchange raises (no rank waits forever), and the
  library's own plan (mrg_run_job / the mrgpu CLI with the RCCL communicator forced on) fails cleanly
  at every injected stage (MRG_TEST_FAIL).
* Exchange records: counts split over several records (MRG_TEST_XREC_VMAX), an import that replaces a
  wide-path map result, and a C5 slice with truncated internal hashes (forced collisions).
"""
import gzip
import hashlib
import json
import os
import subprocess
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
MIB = 1 << 20
THREADS = min(16, os.cpu_count() or 4)   # the GPU box's CPU share is 16
SEED = {"zipf": 0x5EED2026, "unique": 0xC5C5}


def sha(b):
    return hashlib.sha256(b).hexdigest()


def _gen(ctx, kind, file_indices, fbytes):
    import torch
    buf = torch.empty(len(file_indices) * fbytes + 64, dtype=torch.uint8, device="cuda:0")
    for i, fi in enumerate(file_indices):
        p = buf.data_ptr() + i * fbytes
        if kind == "zipf":
            ctx.gen_zipf(p, fbytes, SEED[kind], fi, 1 << 20, 1.1)
        else:
            ctx.gen_unique(p, fbytes, SEED[kind], fi)
    torch.cuda.synchronize()
    return buf


def _rank_main(rank, world, init_file, out_dir, kind, files_per_rank, fbytes, R, fail_rank):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    import torch
    import torch.distributed as dist
    import mapreduce_rust_amd as M
    from mapreduce_rust_amd import shuffle as S
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    res = {}
    with M.Context(0) as c:
        idx = [rank * files_per_rank + i for i in range(files_per_rank)]
        buf = _gen(c, kind, idx, fbytes)
        c.job_begin(M.APP_WC, R)
        c.set_input(buf.data_ptr(), [i * fbytes for i in range(files_per_rank + 1)], idx)
        c.map()
        st = c.stats()
        res["map_distinct"] = st["distinct_keys"]
        res["map_records"] = st["map_records"]
        if rank == fail_rank:
            def broken(n_owners):
                raise M.MrgError(M.native.EINVAL, "injected export failure (test)")
            c.export_sizes = broken
        t0 = time.time()
        try:
            n_rec, n_heap = S.shuffle(c, world, "cuda:0")
        except M.MrgError as e:
            res["error"] = e.code
            res["error_s"] = time.time() - t0
        else:
            res["n_rec"], res["n_heap"] = n_rec, n_heap
            res["import_distinct"] = c.stats()["distinct_keys"]
            c.reduce()
            outs = c.outputs()
            res["sha"] = {str(r): sha(outs[r]) for r in range(R) if r % world == rank}
            res["empty"] = all(outs[r] == b"" for r in range(R) if r % world != rank)
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def _spawn(tmp_path, world, kind, files_per_rank, fbytes, R, fail_rank=-1):
    import torch.multiprocessing as mp
    mp.start_processes(_rank_main, args=(world, str(tmp_path / "init"), str(tmp_path), kind, files_per_rank, fbytes,
                                         R, fail_rank), nprocs=world, join=True, start_method="spawn")
    return [json.load(open(tmp_path / f"rank{rk}.json")) for rk in range(world)]


@pytest.mark.parametrize("kind,world,files_per_rank", [("zipf", 2, 2), ("zipf", 3, 2), ("unique", 2, 3),
                                                       ("unique", 3, 2)])
def test_ranks_exchange_vs_oracle(tmp_path, kind, world, files_per_rank):
    """C4's shape (Zipf(1.1), vocabulary 2^20, 512 MiB per rank) and C5's (near-unique 12-byte keys,
    512-768 MiB per rank: 4e7-6e7 distinct keys per rank, each map taking the wide aggregation) at
    world 2 and 3, nReduce 64: the union of the ranks' owned partitions is byte-identical to the
    oracle over all ranks' bytes."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    fbytes, R = 256 * MIB, 64
    n_files = world * files_per_rank
    with M.Context(0) as ctx:
        buf = _gen(ctx, kind, list(range(n_files)), fbytes)
        host = np.empty(n_files * fbytes, dtype=np.uint8)
        import torch
        torch.from_numpy(host).copy_(buf[:n_files * fbytes])
        del buf
    exp = O.wc_mt([host[i * fbytes:(i + 1) * fbytes] for i in range(n_files)], R, threads=THREADS)
    del host
    exp_sha = [sha(e) for e in exp]
    res = _spawn(tmp_path, world, kind, files_per_rank, fbytes, R)
    merged = {}
    for rk, r in enumerate(res):
        assert "error" not in r, (rk, r)
        assert r["empty"], rk
        merged.update(r["sha"])
        assert r["n_heap"] == 0  # 12-byte and Zipf keys: no long keys, records are 24 bytes each
    assert sorted(int(p) for p in merged) == list(range(R))
    assert [merged[str(p)] for p in range(R)] == exp_sha
    # every key a rank held went out as one record; every rank re-aggregated what it received
    assert sum(r["n_rec"] for r in res) == sum(r["map_distinct"] for r in res)
    if kind == "unique":
        total_import = sum(r["n_rec"] for r in res)
        assert total_import >= 8e7, total_import
        if world == 2:  # >= 5e7 records imported by each rank, through the high-cardinality path
            assert min(r["n_rec"] for r in res) >= 5e7, [r["n_rec"] for r in res]
        # near-unique: the imported distinct keys are the records less the few cross-rank repeats
        assert sum(r["import_distinct"] for r in res) >= 0.99 * total_import
    else:
        # every word once over the owners: the oracle's lines plus each partition's dropped last key
        assert sum(r["import_distinct"] for r in res) == sum(e.count(b"\n") for e in exp) + R


def test_ranks_exchange_rank_failure(tmp_path):
    """Rank 1's export fails: it still joins the counts exchange with a failure status, so rank 0
    raises MRG_ECOMM at once instead of waiting in the data all-to-all, and rank 1 raises its own
    error."""
    import mapreduce_rust_amd as M
    res = _spawn(tmp_path, 2, "zipf", 1, 16 * MIB, 10, fail_rank=1)
    assert res[1]["error"] == M.native.EINVAL, res[1]
    assert res[0]["error"] == M.native.ECOMM, res[0]
    assert res[0]["error_s"] < 60


def _data_dir(tmp_path, docs):
    d = tmp_path / "data"
    d.mkdir(exist_ok=True)
    for m, c in enumerate(docs):
        (d / f"gut-{m}.txt").write_bytes(c)


def _cli(tmp_path, *args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([os.path.join(ROOT, "mapreduce_rust_amd", "lib", "mrgpu")] + [str(a) for a in args],
                          cwd=tmp_path, env=e, capture_output=True, text=True, timeout=120)


@pytest.fixture(scope="module")
def corpus():
    return [gzip.open(os.path.join(HERE, "golden", "corpus", f"gut-{m}.txt.gz")).read() for m in range(6)]


@pytest.mark.parametrize("stage", ["open", "comm", "map", "export", "recv", "reduce", "write"])
def test_run_job_injected_failure_returns(tmp_path, corpus, stage):
    """mrg_run_job with the RCCL communicator forced on (MRG_TEST_FORCE_COMM) and a failure injected at
    each phase (MRG_TEST_FAIL=<stage>:0): the mrgpu CLI exits 1 with the injected message well within
    the timeout (the phases are joined and the exchange agrees on every rank's status before its
    transfers, so no GPU thread is left waiting); without the knob the same run is golden."""
    _data_dir(tmp_path, corpus)
    t0 = time.time()
    p = _cli(tmp_path, 6, 10, "--gpus", 1, env={"MRG_TEST_FORCE_COMM": "1", "MRG_TEST_FAIL": f"{stage}:0"})
    assert p.returncode == 1, (p.returncode, p.stderr)
    assert "injected failure at stage '%s'" % stage in p.stderr, p.stderr
    assert time.time() - t0 < 60
    p = _cli(tmp_path, 6, 10, "--gpus", 1, "--times", env={"MRG_TEST_FORCE_COMM": "1"})
    assert p.returncode == 0, p.stderr
    for r in range(10):
        assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["wc"]["10"][f"mr-{r}.txt"], r
    times = json.loads(p.stderr.strip().splitlines()[-1])
    assert times["input_bytes"] == sum(len(c) for c in corpus) and times["n_gpus"] == 1


@pytest.fixture(scope="module")
def ctx():
    import mapreduce_rust_amd as M
    c = M.Context(0)
    yield c
    c.close()


def _export(ctx, docs, R, n_owners, vmax=None):
    """Map docs, export for n_owners; returns (records, heap, rec_counts, heap_counts) on the host."""
    import torch
    import mapreduce_rust_amd as M
    from gpu_util import to_device
    t, off = to_device(docs)
    ctx.job_begin(M.APP_WC, R)
    ctx.set_input(t.data_ptr(), off)
    ctx.map()
    old = os.environ.get("MRG_TEST_XREC_VMAX")
    if vmax:
        os.environ["MRG_TEST_XREC_VMAX"] = str(vmax)
    try:
        rec, heap = ctx.export_sizes(n_owners)
        drec = torch.empty(max(sum(rec), 1) * M.native.XREC_BYTES, dtype=torch.uint8, device="cuda:0")
        dheap = torch.empty(max(sum(heap), 1), dtype=torch.uint8, device="cuda:0")
        ctx.export(drec.data_ptr(), dheap.data_ptr())
    finally:
        os.environ.pop("MRG_TEST_XREC_VMAX", None)
        if old is not None:
            os.environ["MRG_TEST_XREC_VMAX"] = old
    return drec.cpu(), dheap.cpu(), rec, heap, ctx.stats()["distinct_keys"]


def test_export_count_split_vs_golden(ctx, corpus):
    """A short key's count travels in 32 bits; larger counts are split over several records, which the
    receiver sums.  With the per-record limit lowered to 7 (MRG_TEST_XREC_VMAX), every key seen more
    than 7 times goes out as several records; the import restores the golden output."""
    import torch
    import mapreduce_rust_amd as M
    drec, dheap, rec, heap, distinct = _export(ctx, corpus, 10, 1, vmax=7)
    assert sum(rec) > distinct + 50_000, (sum(rec), distinct)   # ("the": 32735 / 7 records)
    R = drec[:sum(rec) * M.native.XREC_BYTES].to("cuda:0")
    H = torch.cat([dheap[:sum(heap)], torch.zeros(1, dtype=torch.uint8)]).to("cuda:0")
    ctx.job_begin(M.APP_WC, 10)
    ctx.import_(R.data_ptr(), sum(rec), H.data_ptr(), sum(heap), rec, heap)
    ctx.reduce()
    assert [sha(o) for o in ctx.outputs()] == [GOLDEN["wc"]["10"][f"mr-{r}.txt"] for r in range(10)]


def test_import_replaces_wide_map_result(ctx, corpus):
    """A context whose map took the wide (sort-based) aggregation, then imports another job's records
    without exporting its own: the reduce formats the imported keys, not the map result (the import
    releases the wide result)."""
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import to_device
    other = [corpus[4], corpus[5]]
    drec, dheap, rec, heap, _ = _export(ctx, other, 10, 1)
    os.environ["MRG_WIDE"] = "1"
    try:
        t, off = to_device(corpus[:3])
        ctx.job_begin(M.APP_WC, 10)
        ctx.set_input(t.data_ptr(), off)
        ctx.map()                                   # wide result pending
        R = drec[:max(sum(rec), 1) * M.native.XREC_BYTES].to("cuda:0")
        H = torch.cat([dheap[:sum(heap)], torch.zeros(1, dtype=torch.uint8)]).to("cuda:0")
        ctx.import_(R.data_ptr(), sum(rec), H.data_ptr(), sum(heap), rec, heap)
        ctx.reduce()
        got = ctx.outputs()
    finally:
        os.environ.pop("MRG_WIDE", None)
    assert got == O.wc(other, 10, O.FAST)


def test_c5_forced_collisions_vs_oracle(ctx):
    """SURVEY §8(d) C5's forced-collision run: a 512 MiB near-unique slice (4e7 keys, the wide path)
    plus 260 000 distinct keys of 13..30 bytes (16-byte tail records and the long-key fingerprint sort), every internal hash truncated to 20 bits
    (MRG_FLAG_DEBUG_HASH_BITS(20): map-table sets, tail buckets, HBM tables and the long-key
    fingerprints all collide massively); output byte-identical to the oracle, through the LDS-combine
    map and the wide map (MRG_WIDE_MAP=0 / 1)."""
    import random
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    nf, fb = 2, 256 * MIB
    buf = _gen(ctx, "unique", [100, 101], fb)
    rng = random.Random(5)
    alpha = "abcdefghijklmnopqrstuvwxyz0123456789"
    # 13..16-byte keys (the map's 16-byte tail regions, read by the wide path's L1) and long keys
    longs = " ".join("".join(rng.choice(alpha) for _ in range(rng.randint(13, 30))) for _ in range(260_000))
    longs = (longs + "\n").encode()
    host = np.empty(nf * fb + len(longs), dtype=np.uint8)
    torch.from_numpy(host[:nf * fb]).copy_(buf[:nf * fb])
    host[nf * fb:] = np.frombuffer(longs, dtype=np.uint8)
    del buf
    pad = (-(nf * fb + len(longs))) % 16
    t = torch.from_numpy(np.concatenate([host, np.zeros(64 + pad, dtype=np.uint8)])).to("cuda:0")
    off = [0, fb, 2 * fb, 2 * fb + len(longs)]
    runs = []
    saved = os.environ.get("MRG_WIDE_MAP")
    try:
        for wm in ("0", "1"):  # the LDS-combine map + wide aggregation, then the wide map
            os.environ["MRG_WIDE_MAP"] = wm
            ctx.job_begin(M.APP_WC, 64, M.debug_hash_bits(20))
            ctx.set_input(t.data_ptr(), off)
            ctx.map()
            ctx.reduce()
            runs.append((ctx.outputs(), ctx.stats()))
    finally:
        if saved is None:
            os.environ.pop("MRG_WIDE_MAP", None)
        else:
            os.environ["MRG_WIDE_MAP"] = saved
    del t
    exp = O.wc_mt([host[:fb], host[fb:2 * fb], host[2 * fb:]], 64, threads=THREADS)
    for (got, st), kind in zip(runs, (0, 1)):
        assert st["distinct_keys"] > 40_000_000 and st["long_tokens"] >= 150_000, st
        assert st["agg_path"] == 2 and st["map_kind"] == kind, st
        if kind == 0:
            assert st["tail_records_16"] > 30_000, st
        for r in range(64):
            assert got[r] == exp[r], (kind, r)
