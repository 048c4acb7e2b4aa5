"""GPU parity at full size, on the capacity-overflow paths, and across ranks (all through the C ABI).

* C3 at its full 10 GiB (BASELINE.json configs[2]) and a 1 GiB slice of C5 (configs[4]) against the
  multi-threaded C oracle (tests/oracle_lib.wc_mt, FAST mode, run on the host over the same bytes).
* The map's tail-region spill, grow-and-rerun and the aggregation's overflow regrow forced by the
  test knobs MRG_TEST_TAIL_CAP / MRG_TEST_OVF_CAP / MRG_TEST_AGG_OCAP, against the oracle.
* The exchange: the library's RCCL shuffle (mrg_job_shuffle) in a one-rank communicator, the
  mrgpu CLI and mrg_run_job (GPU threads + communicator), a plain-C FFI host (worker_harness.c) and
  two processes on the one GPU exchanging the library's export records over gloo.
Reference for the path: src/mr/worker.rs:65-193, src/app/wc.rs:6-17, src/run.sh:16-20.
"""
import gzip
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
MIB = 1 << 20
THREADS = min(16, os.cpu_count() or 4)   # the GPU box's CPU share is 16


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def ctx():
    import mapreduce_rust_amd as M
    c = M.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def corpus():
    return [gzip.open(os.path.join(HERE, "golden", "corpus", f"gut-{m}.txt.gz")).read() for m in range(6)]


def _generate(ctx, kind, n_files, file_bytes, seed):
    import torch
    buf = torch.empty(n_files * file_bytes + 64, dtype=torch.uint8, device="cuda:0")
    for i in range(n_files):
        p = buf.data_ptr() + i * file_bytes
        if kind == "zipf":
            ctx.gen_zipf(p, file_bytes, seed, i, 1 << 20, 1.1)
        else:
            ctx.gen_unique(p, file_bytes, seed, i)
    torch.cuda.synchronize()
    return buf


def _host_files(buf, n_files, file_bytes):
    """D2H of the generated input, one numpy view per file (no second host copy)."""
    import torch
    host = np.empty(n_files * file_bytes, dtype=np.uint8)
    torch.from_numpy(host).copy_(buf[:n_files * file_bytes])
    return [host[i * file_bytes:(i + 1) * file_bytes] for i in range(n_files)]


def _run_job(ctx, buf, n_files, file_bytes, R):
    import mapreduce_rust_amd as M
    ctx.job_begin(M.APP_WC, R)
    ctx.set_input(buf.data_ptr(), [i * file_bytes for i in range(n_files + 1)])
    ctx.map()
    ctx.reduce()
    return ctx.outputs()


def test_c3_full_size_vs_oracle(ctx):
    """configs[2]: 40 x 256 MiB of Zipf(1.1) text over 2^20 words, nReduce 64 -- every mr-{r}.txt
    byte-identical to the oracle's on the same 10 GiB."""
    import oracle_lib as O
    nf, fb = 40, 256 * MIB
    buf = _generate(ctx, "zipf", nf, fb, 0x5EED2026)
    got = _run_job(ctx, buf, nf, fb, 64)
    st = ctx.stats()
    files = _host_files(buf, nf, fb)
    del buf
    exp = O.wc_mt(files, 64, threads=THREADS)
    assert st["distinct_keys"] == 1 << 20
    assert [sha(g) for g in got] == [sha(e) for e in exp]


def test_c5_slice_vs_oracle(ctx, knobs):
    """configs[4] (1e9 near-unique keys), a 1 GiB slice: 4 x 256 MiB, ~8e7 distinct 12-byte keys.
    (1) The FIRST job of a fresh context -- what every mrg_run_job / one-shot worker call is -- samples
    the input, finds it near-unique and takes the wide map in ONE launch (r06; until r05 the cold job
    ran the LDS-combine map, overflowed and reran it).  (2) A second job on that context: the wide map
    again.  (3) The LDS-combine map with the wide (sort-based) aggregation behind it (MRG_WIDE_MAP=0
    rules the wide map out; the aggregation switches to the wide path by the map's counters).  All
    byte-identical to the oracle."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    nf, fb = 4, 256 * MIB
    buf = _generate(ctx, "unique", nf, fb, 0xC5C5)
    knobs()
    with M.Context(0) as fresh:
        got = _run_job(fresh, buf, nf, fb, 64)
        st = fresh.stats()
        got2 = _run_job(fresh, buf, nf, fb, 64)
        st2 = fresh.stats()
    knobs(MRG_WIDE_MAP=0)
    got3 = _run_job(ctx, buf, nf, fb, 64)
    st3 = ctx.stats()
    knobs()
    files = _host_files(buf, nf, fb)
    del buf
    assert st["distinct_keys"] > 70_000_000
    assert st["map_kind"] == 1 and st["map_launches"] == 1 and st["agg_path"] == 2, st
    assert st2["map_kind"] == 1 and st2["map_launches"] == 1 and st2["distinct_keys"] == st["distinct_keys"]
    assert st3["map_kind"] == 0 and st3["agg_path"] == 2 and st3["distinct_keys"] == st["distinct_keys"], st3
    exp = O.wc_mt(files, 64, threads=THREADS)
    assert len(got) == len(exp) == len(got2) == len(got3)
    for r in range(64):
        assert got[r] == exp[r], r
        assert got2[r] == exp[r], r
        assert got3[r] == exp[r], r


def test_cold_context_zipf_takes_bucket_path_vs_oracle(ctx):
    """The cold-context sample on text with repeats (a 512 MiB Zipf slice of C3): the FIRST job of a
    fresh context samples, finds repeats, and takes the LDS-combine map + bucket aggregation in one map
    launch; byte-identical to the oracle."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    nf, fb = 2, 256 * MIB
    buf = _generate(ctx, "zipf", nf, fb, 0x5EED2026)
    with M.Context(0) as fresh:
        got = _run_job(fresh, buf, nf, fb, 64)
        st = fresh.stats()
        n_alloc, alloc_bytes, alloc_ms = fresh.pool_alloc_stats()
    files = _host_files(buf, nf, fb)
    del buf
    assert st["map_kind"] == 0 and st["agg_path"] == 1 and st["map_launches"] == 1, st
    assert st["spec_agg"] == 1, st   # the aggregation was queued behind the cold job's map and used
    assert n_alloc > 0 and alloc_bytes > 0 and alloc_ms >= 0.0
    exp = O.wc_mt(files, 64, threads=THREADS)
    assert [sha(g) for g in got] == [sha(e) for e in exp]


def test_closed_context_blocks_reused_by_the_next(ctx):
    """The process-wide device cache (mrgpu.cpp DeviceCache): a context closed after a 256 MiB Zipf job
    leaves its device blocks behind, and the next context's first job over the same input allocates
    fewer of them (hipMalloc calls counted by mrg_pool_alloc_stats) and writes the same bytes; every
    job's output against the oracle."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    nf, fb = 1, 256 * MIB
    buf = _generate(ctx, "zipf", nf, fb, 0x5EED2026)
    with M.Context(0) as a:
        got_a = _run_job(a, buf, nf, fb, 16)
        na = a.pool_alloc_stats()[0]
    with M.Context(0) as b:
        got_b = _run_job(b, buf, nf, fb, 16)
        nb = b.pool_alloc_stats()[0]
    files = _host_files(buf, nf, fb)
    del buf
    assert na > 0 and nb < na, (na, nb)
    assert got_a == got_b == O.wc_mt(files, 16, threads=THREADS)


@pytest.mark.parametrize("knob", [{}, {"MRG_TEST_WMAP_CAP": 2}, {"MRG_TEST_WMAP_B1R": 1}, {"MRG_TEST_WMAP_B1R": 3},
                                  {"MRG_TEST_WMAP_W12": 0}, {"MRG_TEST_WMAP_W12": 1, "MRG_TEST_WMAP_L16": 1}])
def test_wide_map_forced_vs_oracle(ctx, corpus, knobs, knob):
    """The wide map forced on (MRG_WIDE_MAP=1): every short key goes from the map straight to its L1
    bucket (SipHash-1-3 partition, then the splitters of a sample of the input), L2 reads the map's
    regions.  C1 golden digests at R = 1/10/64; near-unique, Unicode and long-key documents, and forced
    internal hash collisions, against the oracle.  Knobs: regions of 2 records (every region overflows:
    the launch reruns with regions sized to the demand), one bucket per partition (B1r = 1), three
    (binary splitter search instead of the index), 16-byte regions only (W12=0), and 12-byte regions
    whose lists of 13..16-byte keys hold one record each (the launch reruns with 16-byte regions)."""
    import torch
    import oracle_lib as O
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    knobs(MRG_WIDE_MAP=1, **knob)
    for R in (1, 10, 64):
        outs = run_wc(ctx, corpus, R)
        st = ctx.stats()
        assert st["map_kind"] == 1 and st["agg_path"] == 2, st
        if knob.get("MRG_TEST_WMAP_CAP"):
            assert st["map_launches"] >= 2, st
        assert [sha(o) for o in outs] == [GOLDEN["wc"][str(R)][f"mr-{r}.txt"] for r in range(R)], R
    n = 8 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_unique(t.data_ptr(), n, 0xC5, 3)
    docs = [t[:n].cpu().numpy().tobytes()] + _long_token_docs(5, n_docs=2, n_tokens=20_000) + [
        "naïve café ’tis Ærø ſtraße 東京 — x".encode() * 300, _mixed_keys_doc(11, 50_000)]
    for R in (7, 64):
        exp = O.wc(docs, R, O.FAST)
        assert run_wc(ctx, docs, R) == exp, R
        st = ctx.stats()
        assert st["map_kind"] == 1
        if knob.get("MRG_TEST_WMAP_L16"):
            assert st["map_launches"] >= 2, st
    assert run_wc(ctx, docs, 10, flags=M.debug_hash_bits(4)) == O.wc(docs, 10, O.FAST)


def _rare_byte_keys_doc(seed, n_words=400_000):
    """Near-unique 12-letter keys that share their first bytes, with one key in 2000 taking a byte
    value the rest never use at each of the positions the wide map's L2 digits read: a sample of
    2048 records mostly misses those values, so their digit codes come from the 'value the sample
    lacks' rule (a lacking value collapsed onto a present one, lower bytes kept, reordered keys)."""
    import random
    rng = random.Random(seed)
    common, rare = "abcdefghijklmnop", "z9"
    words = []
    for i in range(n_words):
        w = ["k", "q"] + [rng.choice(common) for _ in range(10)]
        if i % 2000 == 1999:
            for pos in rng.sample(range(1, 6), 2):
                w[pos] = rng.choice(rare)
        words.append("".join(w))
    return " ".join(words).encode()


@pytest.mark.parametrize("b1r", ["1", "4"])
def test_wide_map_rare_byte_values_vs_oracle(ctx, knobs, b1r):
    """The wide map's L2 digit leaves on keys whose rare byte values a bucket's sample misses, at one
    and four quantile buckets per partition, against the oracle (R = 3 and 64)."""
    import oracle_lib as O
    from gpu_util import run_wc
    knobs(MRG_WIDE_MAP=1, MRG_TEST_WMAP_B1R=b1r)
    docs = [_rare_byte_keys_doc(7), _rare_byte_keys_doc(8, 100_000)]
    for R in (3, 64):
        assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST), R
        assert ctx.stats()["map_kind"] == 1


def _mixed_keys_doc(seed, n_words=200_000):
    """Words of 1..16 letters (a few thousand distinct per length) and one word in 100 of 17..20: the
    map's tail records are then a mix of 12-byte records (keys of <= 12 bytes) and 16-byte records
    (13..16 bytes), with a few long keys (fewer than the map's default long-key capacity, so they
    cause no rerun of their own)."""
    import random
    rng = random.Random(seed)
    vocab = ["".join(rng.choice("abcdefghij") for _ in range(L)) for L in range(1, 17) for _ in range(3000)]
    longs = ["".join(rng.choice("abcdefghij") for _ in range(L)) for L in range(17, 21) for _ in range(100)]
    return " ".join(rng.choice(longs) if i % 100 == 99 else rng.choice(vocab) for i in range(n_words)).encode()


@pytest.fixture
def knobs():
    keys = ["MRG_TEST_TAIL_CAP", "MRG_TEST_OVF_CAP", "MRG_TEST_AGG_OCAP", "MRG_WIDE", "MRG_TEST_LEAF_CAP",
            "MRG_TEST_LEAF_TARGET", "MRG_TEST_SORT_LCAP", "MRG_TEST_AGG_WIDE_OVF", "MRG_TEST_AGG_NSUB",
            "MRG_TEST_NO_PACK", "MRG_TEST_LONG_PER", "MRG_TEST_LONG_LIST", "MRG_WIDE_MAP", "MRG_TEST_WMAP_CAP",
            "MRG_TEST_WMAP_B1R", "MRG_TEST_WMAP_W12", "MRG_TEST_WMAP_L16", "MRG_TEST_L2_CAP",
            "MRG_TEST_L2_MIN", "MRG_WIDE_L2_SAMPLED"]
    saved = {k: os.environ.get(k) for k in keys}

    def set_(**kw):
        for k in keys:
            os.environ.pop(k, None)
        for k, v in kw.items():
            os.environ[k] = str(v)
    yield set_
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


@pytest.mark.parametrize("wide", ["0", "1"])
def test_map_spill_and_rerun_vs_oracle(ctx, corpus, knobs, wide):
    """Tail regions of 1 record: (a) records spill into the per-bucket overflow lists (one launch);
    (b) the lists are 16 records too: a launch overflows, regions grow to the measured demand and the
    map reruns.  Both aggregation paths (bucketed / wide) must still equal the oracle."""
    import torch
    import oracle_lib as O
    from gpu_util import run_wc
    n = 16 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_zipf(t.data_ptr(), n, 0x5EED2026, 7, 1 << 16, 1.1)
    docs = corpus[:3] + [t[:n].cpu().numpy().tobytes(), _mixed_keys_doc(1)]
    for R in (10, 64):
        exp = O.wc(docs, R, O.FAST)
        knobs(MRG_TEST_TAIL_CAP=1, MRG_TEST_OVF_CAP=1 << 22, MRG_WIDE=wide)
        assert run_wc(ctx, docs, R) == exp
        st = ctx.stats()
        assert st["map_launches"] == 1 and st["map_spill"] > 100_000, st
        knobs(MRG_TEST_TAIL_CAP=1, MRG_TEST_OVF_CAP=16, MRG_WIDE=wide)
        assert run_wc(ctx, docs, R) == exp
        st = ctx.stats()
        assert st["map_launches"] >= 2 and st["tail_records_16"] > 1000, st
        knobs(MRG_WIDE=wide)                                         # regions sized from the rerun's demand
        assert run_wc(ctx, docs, R) == exp
        assert ctx.stats()["tail_records_16"] > 1000


def test_speculative_aggregation_paths_vs_oracle(ctx, corpus, knobs):
    """The bucket aggregation queued behind the map before the host has read the map's counters
    (mrgpu.cpp job_map): on a context whose previous job took the bucket path it is launched, then
    reused (spec_agg 1) or dropped (spec_agg 2) -- with MRG_WIDE unset, on the map-rerun path
    (tail regions of 1 record, 16-record overflow lists), the aggregation-regrow path (overflow list of
    1000 records, 4-bit hashes) and with sub-ranges; every output against the oracle."""
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import run_wc
    n = 16 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_zipf(t.data_ptr(), n, 0x5EED2026, 9, 1 << 16, 1.1)
    docs = corpus[:3] + [t[:n].cpu().numpy().tobytes()]
    exp = O.wc(docs, 10, O.FAST)

    def primed(**kw):  # a plain job first: it takes the bucket path, so the next job queues the launch
        knobs()
        assert run_wc(ctx, docs, 10) == exp
        assert ctx.stats()["agg_path"] == 1
        knobs(**kw)
        got = run_wc(ctx, docs, 10)
        return got, ctx.stats()

    got, st = primed()
    assert got == exp and st["spec_agg"] == 1 and st["agg_path"] == 1, st
    got, st = primed(MRG_TEST_TAIL_CAP=1, MRG_TEST_OVF_CAP=16)   # map rerun: the queued launch is dropped
    assert got == exp and st["map_launches"] >= 2 and st["spec_agg"] == 2, st
    got, st = primed(MRG_TEST_AGG_NSUB=3)                        # launched with the forced sub-ranges
    assert got == exp and st["spec_agg"] == 1, st
    got, st = primed(MRG_WIDE=0)
    assert got == exp and st["spec_agg"] == 1, st
    knobs()
    run_wc(ctx, corpus, 10, flags=M.debug_hash_bits(4))
    knobs(MRG_TEST_AGG_OCAP=1000)                                # reused, then its overflow list regrown
    got = run_wc(ctx, corpus, 10, flags=M.debug_hash_bits(4))
    st = ctx.stats()
    assert got == O.wc(corpus, 10, O.FAST)
    assert st["spec_agg"] == 1 and st["agg_launches"] >= 2 and st["overflow_keys"] > 1000, st
    knobs(MRG_WIDE=1)                                            # forced wide: nothing queued
    assert run_wc(ctx, docs, 10) == exp
    st = ctx.stats()
    assert st["spec_agg"] == 0 and st["agg_path"] == 2, st


def test_aggregation_overflow_regrow_vs_oracle(ctx, corpus, knobs):
    """Every key in one bucket (4-bit internal hashes), the HBM overflow list of the bucket
    aggregation started at 1000 records: it overflows, is regrown and the aggregation reruns."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import run_wc
    knobs(MRG_TEST_AGG_OCAP=1000, MRG_WIDE=0)
    docs = corpus + [_mixed_keys_doc(3, 50_000)]
    got = run_wc(ctx, docs, 64, flags=M.debug_hash_bits(4))
    st = ctx.stats()
    assert st["agg_launches"] >= 2 and st["overflow_keys"] > 1000 and st["tail_records_16"] > 100, st
    assert got == O.wc(docs, 64, O.FAST)


@pytest.mark.parametrize("lcap", ["1", "48", "2048"])
def test_key_sort_buckets_vs_oracle(ctx, corpus, knobs, lcap):
    """The distinct-key sort (worker.rs:162-164): MSD buckets on (partition bits, leading key bits),
    each bucket bitonic-sorted in LDS, a bucket above MRG_TEST_SORT_LCAP keys sorted by the LSD radix
    sort on its own segment instead (lcap 48: some buckets; lcap 1: more than 16 oversized buckets, so
    the whole array goes through the LSD sort).  R = 20000 leaves one key bit in the bucket id and R = 40000 none
    (buckets = partitions); R = 1 buckets on key bits alone."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import run_wc
    knobs(MRG_TEST_SORT_LCAP=lcap, MRG_WIDE=0)
    for R in (1, 10, 64, 20000, 40000):
        assert run_wc(ctx, corpus, R) == O.wc(corpus, R, O.FAST), R
    # forced internal hash collisions, and the indexer's (word, doc) keys through the same sort
    assert run_wc(ctx, corpus, 10, flags=M.debug_hash_bits(4)) == O.wc(corpus, 10, O.FAST)
    names = [f"data/gut-{m}.txt" for m in range(6)]
    assert run_wc(ctx, corpus, 10, app=M.APP_INDEXER, names=names) == O.indexer(corpus, names, 10)


@pytest.mark.parametrize("nsub", ["2", "3", "16"])
def test_bucket_subranges_vs_oracle(ctx, corpus, knobs, nsub):
    """Every bucket summed by nsub workgroups, each reading all of the bucket's records and keeping
    one hash sub-range (the path of buckets with more distinct keys than one LDS table holds)."""
    import torch
    import oracle_lib as O
    from gpu_util import run_wc
    n = 8 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_zipf(t.data_ptr(), n, 0x5EED2026, 3, 1 << 18, 1.1)
    docs = corpus + [t[:n].cpu().numpy().tobytes(), _mixed_keys_doc(2)]
    knobs(MRG_TEST_AGG_NSUB=nsub, MRG_WIDE=0)
    for R in (10, 64):
        assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST)


def test_bucket_overflow_falls_back_to_wide_vs_oracle(ctx, corpus, knobs):
    """Far more keys missing the per-bucket LDS tables than the overflow path handles well (every
    key in 16 buckets through 4-bit internal hashes; threshold lowered from 4 Mi overflow records to
    100): the bucket aggregation splits buckets over up to 16 workgroups each, still overflows, and
    gives up: the wide (sort-based) aggregation runs on the same map output.  Output equals the
    oracle's."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import run_wc
    knobs(MRG_TEST_AGG_WIDE_OVF=100)
    for R in (1, 10):
        got = run_wc(ctx, corpus, R, flags=M.debug_hash_bits(4))
        assert ctx.stats()["agg_launches"] == 0  # no completed bucket aggregation: the wide path ran
        assert got == O.wc(corpus, R, O.FAST), R


def _long_token_docs(seed, n_docs=6, n_tokens=60_000):
    """Text where about a third of the tokens have keys of more than 16 bytes: em-dash-joined word
    pairs (the long tokens of Gutenberg text), long Unicode words, a few hundred distinct each."""
    import random
    rng = random.Random(seed)
    short = ["the", "of", "and", "wine", "don\u2019t", "caf\u00e9"]
    longs = ["".join(rng.choice("abcdefghij") for _ in range(rng.randint(17, 40))) for _ in range(300)]
    longs += [a + "\u2014" + b for a, b in zip(rng.choices(short + longs[:20], k=200), rng.choices(longs, k=200))]
    longs += ["\u017f" * 9 + "x" for _ in range(3)]   # 19 key bytes of 2-byte letters
    docs = []
    for _ in range(n_docs):
        toks = [rng.choice(longs) if rng.random() < 0.35 else rng.choice(short) for _ in range(n_tokens)]
        docs.append(" ".join(toks).encode())
    return docs


@pytest.mark.parametrize("per,lst", [(0, 0), (1, 100_000), (1, 3)])
def test_long_token_regions_vs_oracle(ctx, knobs, per, lst):
    """Long tokens (keys > 16 bytes) go to the map workgroup's own region through an LDS cursor; a full
    region spills into the shared list (MRG_TEST_LONG_PER=1: every workgroup's second long token), a full
    list reruns the launch with regions grown to the measured demand (MRG_TEST_LONG_LIST=3).  The
    regions are packed densely after the map: wc and indexer outputs equal the oracle's."""
    import oracle_lib as O
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    docs = _long_token_docs(per * 7 + lst)
    knobs(**({"MRG_TEST_LONG_PER": per, "MRG_TEST_LONG_LIST": lst} if per else {}))
    for R in (1, 10):
        assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST), R
        st = ctx.stats()
        assert st["long_tokens"] > 50_000
        if lst == 3:
            assert st["map_launches"] >= 2
    names = [f"data/gut-{m}.txt" for m in range(len(docs))]
    assert run_wc(ctx, docs, 10, app=M.APP_INDEXER, names=names) == O.indexer(docs, names, 10)


def test_library_shuffle_single_rank(ctx, corpus):
    """mrg_job_shuffle (RCCL inside libmrgpu.so) in a one-rank communicator: the counts all-to-all,
    the own-slice copy and the import run; output = golden, no peer bytes."""
    import mapreduce_rust_amd as M
    from gpu_util import to_device
    comm = M.Comm(ctx, M.comm_id(), 1, 0)
    try:
        for R in (10, 64):
            t, off = to_device(corpus)
            ctx.set_timing(True)
            ctx.job_begin(M.APP_WC, R)
            ctx.set_input(t.data_ptr(), off)
            ctx.map()
            ctx.shuffle(comm)
            ctx.reduce()
            outs = ctx.outputs()
            st = ctx.stats()
            ctx.set_timing(False)
            assert [sha(o) for o in outs] == [GOLDEN["wc"][str(R)][f"mr-{r}.txt"] for r in range(R)]
            assert st["exchange_sent"] == 0 and st["exchange_recv"] == 0 and st["ms_exchange"] >= 0.0
            assert st["tokens"] == sum(GOLDEN["corpus"]["tokens"])
    finally:
        comm.close()


def test_shuffle_failure_inside_group_releases_buffers(ctx, corpus):
    """An RCCL failure inside the exchange's send/recv group (MRG_TEST_FAIL=sendrecv: raised after the
    timing events and all four exchange buffers exist) aborts the communicator and fails the call with
    MRG_ECOMM; the context's pool gets every exchange buffer back (mrg_pool_stats' outstanding count is
    the pre-exchange one) and the same context then runs a normal job to the golden output."""
    import mapreduce_rust_amd as M
    from gpu_util import to_device
    comm = M.Comm(ctx, M.comm_id(), 1, 0)
    try:
        assert comm.count() == 1
        t, off = to_device(corpus)
        ctx.job_begin(M.APP_WC, 10)
        ctx.set_input(t.data_ptr(), off)
        ctx.map()
        before = ctx.pool_stats()[0]
        os.environ["MRG_TEST_FAIL"] = "sendrecv"
        try:
            with pytest.raises(M.MrgError) as ei:
                ctx.shuffle(comm)
        finally:
            os.environ.pop("MRG_TEST_FAIL", None)
        assert ei.value.code == -6 and "sendrecv" in str(ei.value), ei.value
        assert ctx.pool_stats()[0] == before
        with pytest.raises(M.MrgError):        # the communicator stays aborted
            comm.count()
        ctx.job_begin(M.APP_WC, 10)
        ctx.set_input(t.data_ptr(), off)
        ctx.map()
        ctx.reduce()
        assert [sha(o) for o in ctx.outputs()] == [GOLDEN["wc"]["10"][f"mr-{r}.txt"] for r in range(10)]
    finally:
        comm.close()


def _data_dir(tmp_path, corpus, extra=None):
    d = tmp_path / "data"
    d.mkdir()
    for m, c in enumerate(corpus + (extra or [])):
        (d / f"gut-{m}.txt").write_bytes(c)


def _cli(tmp_path, *args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([os.path.join(ROOT, "mapreduce_rust_amd", "lib", "mrgpu")] + [str(a) for a in args],
                          cwd=tmp_path, env=e, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize("force_comm", ["0", "1"])
def test_mrgpu_cli_binary(tmp_path, corpus, force_comm):
    """The mrgpu binary (no Python on the data path): `mrgpu 6 10 --gpus 1 --final` in a directory
    holding data/gut-{m}.txt writes the golden mr-{r}.txt and final.txt.  force_comm=1 runs the
    multi-GPU plan's code (GPU thread + RCCL communicator + mrg_job_shuffle) with one GPU."""
    _data_dir(tmp_path, corpus)
    p = _cli(tmp_path, 6, 10, "--gpus", 1, "--final", env={"MRG_TEST_FORCE_COMM": force_comm})
    assert p.returncode == 0, p.stderr
    for r in range(10):
        assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["wc"]["10"][f"mr-{r}.txt"], r
    assert sha((tmp_path / "final.txt").read_bytes()) == GOLDEN["wc"]["10"]["final.txt"]


def test_mrgpu_cli_indexer_and_errors(tmp_path, corpus):
    _data_dir(tmp_path, corpus, extra=[b"fine words \xe2\x82 broken"])
    p = _cli(tmp_path, 6, 10, "--app", "indexer", env={"MRG_TEST_FORCE_COMM": "1"})
    assert p.returncode == 0, p.stderr
    for r in range(10):
        assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["indexer"]["10"][f"mr-{r}.txt"], r
    p = _cli(tmp_path, 7, 10, env={"MRG_TEST_FORCE_COMM": "1"})   # file 6 is not UTF-8 (worker.rs:75 panics)
    assert p.returncode == 1 and "UTF-8" in p.stderr, p.stderr
    p = _cli(tmp_path, 8, 10)                                       # data/gut-7.txt is missing
    assert p.returncode == 1 and "gut-7" in p.stderr, p.stderr
    p = _cli(tmp_path, 6, 10, "--gpus", 64)
    assert p.returncode == 1 and "n_gpus" in p.stderr, p.stderr


def test_ffi_c_host_worker_calls(tmp_path, corpus):
    """A plain-C host making the calls Worker::map / Worker::reduce would make through an FFI crate
    (mrg_map per file, then mrg_reduce per partition; worker.rs:142-193): golden mr-{r}.txt."""
    _data_dir(tmp_path, corpus)
    exe = os.path.join(HERE, "ffi", "build", "worker_harness")
    for R in (10, 3):
        p = subprocess.run([exe, "6", str(R)], cwd=tmp_path, capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr
        for r in range(R):
            assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["wc"][str(R)][f"mr-{r}.txt"], (R, r)
    p = subprocess.run([exe, "6", "10", "--indexer"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    for r in range(10):
        assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["indexer"]["10"][f"mr-{r}.txt"], r


def _rank_main(rank, world, init_file, out_dir):
    """One rank of a 2-process job on the one GPU: the library's map, export and import, the records
    moved by torch.distributed gloo (host staged: RCCL does not put two ranks on one device)."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    import torch
    import torch.distributed as dist
    import mapreduce_rust_amd as M
    from mapreduce_rust_amd import shuffle as S
    from gpu_util import to_device
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    corpus = [gzip.open(os.path.join(HERE, "golden", "corpus", f"gut-{m}.txt.gz")).read() for m in range(6)]
    res = {}
    with M.Context(0) as c:
        for R in (10, 64):
            mine = S.shard_files(len(corpus), rank, world)
            t, off = to_device([corpus[m] for m in mine])
            c.job_begin(M.APP_WC, R)
            c.set_input(t.data_ptr(), off, mine)
            c.map()
            n_rec, _ = S.shuffle(c, world, "cuda:0")
            c.reduce()
            outs = c.outputs()
            res[str(R)] = {str(r): sha(outs[r]) for r in range(R) if r % world == rank}
            res[str(R) + "_empty"] = all(outs[r] == b"" for r in range(R) if r % world != rank)
            res[str(R) + "_n_rec"] = n_rec
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def test_two_ranks_library_exchange(tmp_path):
    """C4's structure at world size 2: each rank maps its files (m % 2), mrg_job_export ->
    all-to-all -> mrg_job_import, reduces the partitions it owns (r % 2); the union is golden."""
    import torch.multiprocessing as mp
    mp.start_processes(_rank_main, args=(2, str(tmp_path / "init"), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    merged = {"10": {}, "64": {}}
    for rk in range(2):
        res = json.load(open(tmp_path / f"rank{rk}.json"))
        for R in ("10", "64"):
            merged[R].update(res[R])
            assert res[R + "_empty"] and res[R + "_n_rec"] > 0
    for R in ("10", "64"):
        assert sorted(int(r) for r in merged[R]) == list(range(int(R)))
        for r in range(int(R)):
            assert merged[R][str(r)] == GOLDEN["wc"][R][f"mr-{r}.txt"], (R, r)


@pytest.mark.parametrize("wmap", ["0", "1"])
@pytest.mark.parametrize("cap,target", [("0", "1024"), ("8", "1024"), ("0", "16"), ("64", "100000")])
def test_wide_sample_sort_knobs_vs_oracle(ctx, corpus, knobs, cap, target, wmap):
    """The wide aggregation (k_wide.hip) with its leaf capacity / leaf size knobs: cap 8 sends most
    leaves to the global-sort fallback, target 16 makes thousands of tiny leaves, target 100000 one
    leaf per L1 bucket (its distinct keys overflow a 64-key cap).  Inputs: near-unique keys, Zipf
    (hot keys come through the flushed map tables as weighted keys), the corpus, long keys.  wmap=1:
    the same through the wide map, whose L2 cuts leaves from byte-code digits (hot keys: digits of
    many equal keys, leaves past the cap)."""
    import torch
    import oracle_lib as O
    from gpu_util import run_wc
    n = 4 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_unique(t.data_ptr(), n, 0xC5, 9)
    uniq = t[:n].cpu().numpy().tobytes()
    ctx.gen_zipf(t.data_ptr(), n, 0x5EED2026, 3, 1 << 14, 1.1)
    zipf = t[:n].cpu().numpy().tobytes()
    knobs(MRG_WIDE=1, MRG_TEST_LEAF_CAP=cap, MRG_TEST_LEAF_TARGET=target, MRG_WIDE_MAP=wmap)
    for docs, R in (([uniq], 16), ([zipf, uniq[:MIB]], 7), (corpus, 10), ([uniq, b"x" * 40 + b" y"], 3)):
        assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST), (len(docs), R)
    if cap == "8" and wmap == "0":
        assert ctx.stats()["overflow_keys"] > 0   # leaves finished by the fallback


@pytest.mark.parametrize("nopack", ["0", "1"])
def test_wide_packed_counts_vs_oracle(ctx, knobs, nopack):
    """One-wave leaves whose keys are all <= 12 bytes store their counts in the key slots' low word
    (k_wide.hip, packed leaves); leaves holding a 13..16-byte key, workgroup and fallback leaves keep
    the count array.  Near-unique 12-byte keys with 13..16-byte words and repeated keys mixed in,
    packed and (MRG_TEST_NO_PACK) unpacked, through the line writer and through the dense key set
    (final.txt), against the oracle."""
    import torch
    import oracle_lib as O
    from gpu_util import run_wc
    n = 4 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_unique(t.data_ptr(), n, 0xC5, 13)
    uniq = t[:n].cpu().numpy().tobytes()
    longw = b" ".join(b"w%013d" % i + b"q" * (i % 3) for i in range(20000))  # 14..16-byte keys
    reps = b" ".join([b"repeated"] * 5000 + [b"twelvecharsx"] * 3000)
    knobs(MRG_WIDE=1, MRG_TEST_NO_PACK=nopack)
    for docs, R in (([uniq], 16), ([uniq[: 2 * MIB], longw, reps], 7), ([reps, uniq[:MIB]], 1)):
        assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST), (len(docs), R)
    # the dense key set made from the leaves (final.txt, built on the device from the job's keys):
    # LC_ALL=C sort of every mr-{r}.txt line (src/run.sh:16-20)
    docs = [uniq[:MIB], longw, reps]
    outs = run_wc(ctx, docs, 5)
    assert outs == O.wc(docs, 5, O.FAST)
    assert ctx.final() == b"".join(l + b"\n" for l in sorted(l for o in outs for l in o.split(b"\n") if l))


def test_wide_many_partitions_vs_oracle(ctx, knobs):
    """R > 4096 takes the radix-sort form of the wide aggregation (the L1 histogram is per-LDS)."""
    import torch
    import oracle_lib as O
    from gpu_util import run_wc
    n = 2 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_unique(t.data_ptr(), n, 0xC5, 11)
    docs = [t[:n].cpu().numpy().tobytes()]
    knobs(MRG_WIDE=1)
    for R in (5000, 4096):
        assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST), R


def test_wide_l2_sampled_leaves_vs_oracle(ctx, knobs):
    """The wide map's sampled L2 (MRG_WIDE_L2_SAMPLED; k_wide.hip k_wl2): a
    bucket's digit histogram from a quarter of its records, fixed-capacity leaf regions, and the exact
    second launch for every bucket whose leaf overflowed.  256 MiB of near-unique keys at R = 16 (every bucket sampled: the size floor
    lowered to 1024 records), then mixed lengths and repeated keys at R = 7; default capacities, regions
    of 1 x the sampled count (every bucket overflows: all redone), 3 x (some redone), and the exact
    histogram (the default) -- all byte-identical to the oracle."""
    import torch
    import oracle_lib as O
    from gpu_util import run_wc
    nf, fb = 1, 256 * MIB
    buf = _generate(ctx, "unique", nf, fb, 0x15A3)
    files = _host_files(buf, nf, fb)
    exp = O.wc_mt(files, 16, threads=THREADS)
    docs = [_mixed_keys_doc(13, 300_000), b" ".join([b"repeated"] * 40000 + [b"twelvecharsx"] * 30000)]
    exp2 = O.wc(docs, 7, O.FAST)
    sampled = {"MRG_WIDE_L2_SAMPLED": 1}
    for knob in (sampled, dict(sampled, MRG_TEST_L2_CAP="1,0"), dict(sampled, MRG_TEST_L2_CAP="3,0"), {}):
        knobs(MRG_WIDE_MAP=1, MRG_TEST_L2_MIN=1024, **knob)
        got = _run_job(ctx, buf, nf, fb, 16)
        st = ctx.stats()
        assert st["map_kind"] == 1 and st["agg_path"] == 2, (knob, st)
        assert [sha(g) for g in got] == [sha(e) for e in exp], knob
        knobs(MRG_WIDE_MAP=1, MRG_TEST_L2_MIN=64, **knob)
        assert run_wc(ctx, docs, 7) == exp2, knob
    knobs()
    del buf


def test_zipf_unicode_256mib_vs_oracle(ctx):
    """The C3 text with Gutenberg-like Unicode (bench --workload zipf_u: U+2019 apostrophes, U+201C/D
    quotes, U+2014 joining words, U+00E9 letters) -- 256 MiB, nearly every 1 KiB tile non-ASCII, R = 64:
    byte-identical to the oracle (wc.rs:7-10 is Unicode-exact)."""
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    n = 256 * MIB
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_text(t.data_ptr(), n, 0x5EED2026, 3, 1 << 20, 1.1, 1)
    torch.cuda.synchronize()
    host = np.empty(n, dtype=np.uint8)
    torch.from_numpy(host).copy_(t[:n])
    ctx.job_begin(M.APP_WC, 64)
    ctx.set_input(t.data_ptr(), [0, n])
    ctx.map()
    ctx.reduce()
    got = ctx.outputs()
    st = ctx.stats()
    del t
    assert st["nonascii_tiles"] > 0.9 * (n // 1024), st
    exp = O.wc_mt([host], 64, threads=THREADS)
    assert [sha(g) for g in got] == [sha(e) for e in exp]
