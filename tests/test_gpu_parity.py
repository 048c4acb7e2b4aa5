"""GPU parity: libmrgpu.so (HIP, gfx950) against the committed golden digests and the C oracle.

Bar: bit-exact mr-{r}.txt bytes.  Everything goes through the C ABI (mapreduce_rust_amd.native).
"""
import gzip
import hashlib
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
X = 24  # exchange record bytes (include/mrgpu.h MRG_XREC_BYTES)


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


@pytest.mark.parametrize("R", ["10", "1", "3", "64"])
def test_c1_wc_golden(ctx, corpus, R):
    from gpu_util import run_wc
    outs = run_wc(ctx, corpus, int(R))
    g = GOLDEN["wc"][R]
    bad = [r for r in range(int(R)) if sha(outs[r]) != g[f"mr-{r}.txt"]]
    assert not bad, f"partitions differ: {bad}"
    st = ctx.stats()
    assert st["tokens"] == sum(GOLDEN["corpus"]["tokens"])


def test_c1_matches_oracle_bytes(ctx, corpus):
    import oracle_lib as O
    from gpu_util import run_wc
    outs = run_wc(ctx, corpus, 10)
    exp = O.wc(corpus, 10, O.FAST)
    for r in range(10):
        assert outs[r] == exp[r], r


def test_c2_indexer_golden(ctx, corpus):
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    names = [f"data/gut-{m}.txt" for m in range(6)]
    outs = run_wc(ctx, corpus, 10, app=M.APP_INDEXER, names=names)
    for r in range(10):
        assert sha(outs[r]) == GOLDEN["indexer"]["10"][f"mr-{r}.txt"], r


def test_tokenizer_kats(ctx):
    """Each KAT input as a one-document job, R=1, last group kept: lines = sorted distinct tokens."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import run_wc
    for case in GOLDEN["tokenizer"]:
        data = case["input"].encode()
        outs = run_wc(ctx, [data], 1, flags=M.FLAG_NO_COMPAT_DROP_LAST)
        counts = {}
        for t in case["tokens"]:
            counts[t.encode()] = counts.get(t.encode(), 0) + 1
        exp = b"".join(k + b" " + str(v).encode() + b"\n" for k, v in sorted(counts.items()))
        assert outs[0] == exp, case["input"]
        assert O.wc([data], 1)[0] == run_wc(ctx, [data], 1)[0]


def test_invalid_utf8_is_an_error(ctx):
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    for bad in [b"\xff", b"ab\xc0\x80 cd", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"abc \xe2\x82", b"\x80x",
                b"x" * 5000 + b"\xe2\x82" + b" y" * 10, b"a" * 4095 + b"\xa9"]:
        with pytest.raises(M.MrgError) as ei:
            run_wc(ctx, [b"fine text", bad], 3)
        assert ei.value.code == -2


def test_dense_invalid_bytes_then_reuse(ctx):
    """Binary-like documents (KiBs of 0xFF, of 0xC3 leads without continuations, of 0xE2 0x80 pairs)
    between valid ones: every codepoint-lead byte counts as a lead, so a 1 KiB tile can hold up to 1 KiB
    of them -- more than the UTF-8 class path's queue takes (k_map.hip QCAP).  The job must fail with
    MRG_EUTF8 (the reference's read_to_string panic, worker.rs:75), and the same context must then run a
    valid job exactly (no LDS or tail-cursor corruption left behind)."""
    import oracle_lib as O
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    good = [b"fine text " * 300, "café naïve ’tis ".encode() * 200]
    for junk in [b"\xff" * 3000, b"\xc3" * 4096, b"\xe2\x80" * 2500, b"\xf0" * 2100 + b"abc",
                 b"ok " * 700 + b"\xc3" * 2048 + b" ok"]:
        for R in (1, 10):
            with pytest.raises(M.MrgError) as ei:
                run_wc(ctx, [good[0], junk, good[1]], R)
            assert ei.value.code == -2
        docs = good + [b"after the error " * 500]
        assert run_wc(ctx, docs, 10) == O.wc(docs, 10, O.FAST)


def _rand_text(rng, n_tokens, alphabet, seps, max_len=30):
    out = []
    for _ in range(n_tokens):
        L = rng.randint(1, max_len)
        out.append("".join(rng.choice(alphabet) for _ in range(L)))
        out.append(rng.choice(seps))
    return "".join(out).encode("utf-8")


ALPHA = list("abcdeXYZ09_") + ["é", "ß", "ж", "中", "̸", "‍", "'", "-", "’", ".", "\u001c", "😀", "²", "ſ", "Å"]
SEPS = [" ", "\n", "\t", " ", " ", "　", " ", "\u0085", "  ", "\r\n"]


@pytest.mark.parametrize("seed", range(6))
def test_random_unicode_vs_oracle(ctx, seed):
    import oracle_lib as O
    from gpu_util import run_wc
    rng = random.Random(seed)
    docs = [_rand_text(rng, rng.randint(0, 3000), ALPHA[: 6 + seed * 3], SEPS, max_len=[5, 12, 40][seed % 3])
            for _ in range(rng.randint(1, 5))]
    for R in (1, 7):
        assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST)


@pytest.mark.parametrize("gap", [7, 24, 31, 32, 33, 48, 120])
def test_codepoint_density_sweep_vs_oracle(ctx, gap):
    """One non-ASCII codepoint every ~`gap` bytes: a 2 KiB block holds ~2048/gap codepoint leads, so
    the sweep crosses k_map's compacted decode (a lane with 2+ leads, at most 64 leads per block, one
    per lane) and the per-lane loop it falls back to above 64.  Codepoints of 2, 3 and 4 bytes, word
    and White_Space classes, leads placed at every offset of a 16-byte lane segment; then one
    invalid sequence per document at a few densities (MRG_EUTF8)."""
    import oracle_lib as O
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    rng = random.Random(gap)
    cps = ["é", "ж", "’", "—", "“", "中", "😀", " ", "　", "ſ", "ß"]
    def doc(n):
        out, L = [], 0
        while L < n:
            w = "".join(rng.choice("abcdefgh") for _ in range(rng.randint(1, gap)))
            c = rng.choice(cps)
            s = w + c + rng.choice([" ", "", "\n"])
            out.append(s)
            L += len(s.encode())
        return "".join(out).encode()
    docs = [doc(rng.randint(3000, 40000)) for _ in range(4)]
    for R in (1, 7):
        assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST)
    if gap in (24, 32, 48):
        d = bytearray(docs[1])
        d[len(d) // 2] = 0xE2  # a lead without its continuations (or a broken one) mid-document
        d[len(d) // 2 + 1] = 0x41
        with pytest.raises(M.MrgError) as ei:
            run_wc(ctx, [docs[0], bytes(d)], 3)
        assert ei.value.code == -2
        assert run_wc(ctx, docs, 3) == O.wc(docs, 3, O.FAST)


@pytest.mark.parametrize("steal", ["2", "16"])
def test_map_block_pool_vs_oracle(ctx, corpus, steal):
    """k_map's pool of blocks (mrgpu.cpp map_steal) on inputs below its size
    floor (MRG_TEST_STEAL_MIN=0): half (steal = 2) or 1/16 of the blocks taken from the 8 part counters
    by workgroups done with their share -- C1 golden digests, the indexer golden, Unicode and long
    tokens, deferred (invalid) UTF-8 and a near-unique document through the wide map, against the
    oracle; a pooled block with invalid UTF-8 fails the job like any other."""
    import oracle_lib as O
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    keys = ("MRG_MAP_STEAL", "MRG_TEST_STEAL_MIN", "MRG_WIDE_MAP")
    saved = {k: os.environ.get(k) for k in keys}
    os.environ["MRG_MAP_STEAL"] = steal
    os.environ["MRG_TEST_STEAL_MIN"] = "0"
    try:
        for R in ("10", "64"):
            outs = run_wc(ctx, corpus, int(R))
            assert [sha(o) for o in outs] == [GOLDEN["wc"][R][f"mr-{r}.txt"] for r in range(int(R))], R
        names = [f"data/gut-{m}.txt" for m in range(6)]
        outs = run_wc(ctx, corpus, 10, app=M.APP_INDEXER, names=names)
        assert [sha(o) for o in outs] == [GOLDEN["indexer"]["10"][f"mr-{r}.txt"] for r in range(10)]
        rng = random.Random(int(steal))
        docs = [_rand_text(rng, 20000, ALPHA, SEPS, max_len=40) for _ in range(3)] + corpus[:2]
        for R in (1, 7):
            assert run_wc(ctx, docs, R) == O.wc(docs, R, O.FAST), R
        bad = bytearray(corpus[3])
        bad[len(bad) - 3000] = 0xC3  # a lead without its continuation near the end: a pooled block
        bad[len(bad) - 2999] = 0x41
        with pytest.raises(M.MrgError) as ei:
            run_wc(ctx, [corpus[0], bytes(bad)], 3)
        assert ei.value.code == -2
        assert run_wc(ctx, docs, 7) == O.wc(docs, 7, O.FAST)
        import torch
        n = 8 << 20
        t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
        ctx.gen_unique(t.data_ptr(), n, 0xC5, 5)
        udoc = [t[:n].cpu().numpy().tobytes()]
        os.environ["MRG_WIDE_MAP"] = "1"
        assert run_wc(ctx, udoc, 64) == O.wc(udoc, 64, O.FAST)
        assert ctx.stats()["map_kind"] == 1
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_tile_boundaries_and_long_tokens(ctx):
    """Tokens straddling 4 KiB tiles / 16 B lane segments / the 256 B halo, and > 16 B keys."""
    import oracle_lib as O
    from gpu_util import run_wc
    rng = random.Random(7)
    parts = []
    for i in range(3000):
        L = rng.choice([1, 2, 15, 16, 17, 31, 300, 700, 5000])
        parts.append(("k%d" % (i % 50)) * (L // 3 + 1))
        parts.append(rng.choice([" ", "-", " ", "\n", "’", "é "]))
    data = "".join(parts).encode()
    for R in (1, 5):
        assert run_wc(ctx, [data], R) == O.wc([data], R, O.FAST)


def test_document_offsets_and_tile_edges(ctx):
    """Documents starting at every offset mod 16, with words ending exactly on 1 KiB tile and 2 KiB
    block edges (a start at a tile's first byte takes the previous tile's last class)."""
    import oracle_lib as O
    from gpu_util import run_wc
    unit = b"five six seven "  # 15 bytes: word/space phases cycle through every tile alignment
    for lead in range(16):
        d0 = (b"ab " * 800)[:lead + 16 * 37]
        docs = [d0, unit * 150, b"".join(b"w%03da w%03db " % (i, i) for i in range(200)), unit * 3]
        exp = O.wc(docs, 3, O.FAST)
        assert run_wc(ctx, docs, 3) == exp, lead


@pytest.mark.parametrize("bits", [1, 4, 12, 20])
def test_forced_hash_collisions(ctx, corpus, bits):
    """Truncated internal hashes (every key in a few buckets and fingerprint runs): the output must
    still equal the oracle's (collision-safe tie-breaks, the bucket aggregation's HBM overflow)."""
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import run_wc
    docs = corpus[:2] + [("".join("longprefix_shared_%05d " % (i % 700) for i in range(6000))).encode()]
    exp = O.wc(docs, 10, O.FAST)
    got = run_wc(ctx, docs, 10, flags=M.debug_hash_bits(bits))
    assert got == exp
    if bits <= 4:
        assert ctx.stats()["overflow_keys"] > 0   # keys past a bucket's LDS table: the exact HBM path ran


def test_empty_inputs(ctx):
    from gpu_util import run_wc
    assert run_wc(ctx, [b""], 4) == [b""] * 4
    assert run_wc(ctx, [b"   \n\t "], 2) == [b""] * 2
    assert run_wc(ctx, [b"a a a"], 1) == [b""]
    assert run_wc(ctx, [b"b a a c"], 1) == [b"a 2\nb 1\n"]


def test_plugin_surface_map_reduce(ctx, corpus):
    """mrg_map per file + mrg_reduce per partition == the whole job (worker.rs task structure)."""
    import mapreduce_rust_amd as M
    parts = [ctx.map_task(M.APP_WC, corpus[m], f"data/gut-{m}.txt", m, 10) for m in range(6)]
    for r in range(10):
        out = ctx.reduce_task(M.APP_WC, r, parts, 10)
        assert sha(out) == GOLDEN["wc"]["10"][f"mr-{r}.txt"], r
    for p in parts:
        p.free()


def test_two_owner_exchange_on_one_gpu(ctx, corpus):
    """Static plan with 2 owners (r % 2): two map shards exported, cross-imported, reduced."""
    import torch
    import mapreduce_rust_amd as M
    from gpu_util import to_device
    shards = [corpus[0:3], corpus[3:6]]
    sends = []
    for sh in shards:
        t, off = to_device(sh)
        ctx.job_begin(M.APP_WC, 10)
        ctx.set_input(t.data_ptr(), off)
        ctx.map()
        rec, heap = ctx.export_sizes(2)
        drec = torch.empty(max(sum(rec), 1) * X, dtype=torch.uint8, device="cuda:0")
        dheap = torch.empty(max(sum(heap), 1), dtype=torch.uint8, device="cuda:0")
        ctx.export(drec.data_ptr(), dheap.data_ptr())
        sends.append((drec.cpu(), dheap.cpu(), rec, heap))
    outs = {}
    for owner in range(2):
        recs, heaps, sr, sh = [], [], [], []
        for drec, dheap, rec, heap in sends:
            ro = sum(rec[:owner]) * X
            ho = sum(heap[:owner])
            recs.append(drec[ro:ro + rec[owner] * X])
            heaps.append(dheap[ho:ho + heap[owner]])
            sr.append(rec[owner])
            sh.append(heap[owner])
        R = torch.cat(recs).to("cuda:0")
        H = torch.cat(heaps + [torch.zeros(1, dtype=torch.uint8)]).to("cuda:0")
        ctx.job_begin(M.APP_WC, 10)
        ctx.import_(R.data_ptr(), sum(sr), H.data_ptr(), sum(sh), sr, sh)
        ctx.reduce()
        o = ctx.outputs()
        for r in range(10):
            if r % 2 == owner:
                outs[r] = o[r]
            else:
                assert o[r] == b""
    for r in range(10):
        assert sha(outs[r]) == GOLDEN["wc"]["10"][f"mr-{r}.txt"], r


def test_rccl_shuffle_single_rank(tmp_path, corpus):
    """The product exchange (shuffle.shuffle over RCCL all-to-all) in a one-rank nccl group: the
    job's own records go out and come back through the collective, output = golden; the exchange's
    event timing (bench.py's xGMI roofline) is recorded with zero peer bytes."""
    import torch
    import torch.distributed as dist
    import mapreduce_rust_amd as M
    from mapreduce_rust_amd import shuffle as S
    from gpu_util import to_device
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"file://{tmp_path}/pg", rank=0, world_size=1, device_id=dev)
    c = M.Context(0)
    try:
        c.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        t, off = to_device(corpus)
        S.EXCHANGES.clear()
        c.job_begin(M.APP_WC, 10)
        c.set_input(t.data_ptr(), off)
        c.map()
        n_rec, _ = S.shuffle(c, 1, dev)
        c.reduce()
        outs = c.outputs()
        torch.cuda.synchronize(dev)
        assert n_rec > 0
        for r in range(10):
            assert sha(outs[r]) == GOLDEN["wc"]["10"][f"mr-{r}.txt"], r
        assert len(S.EXCHANGES) == 1
        e = S.EXCHANGES[0]
        assert e["sent"] == 0 and e["received"] == 0
        assert e["start"].elapsed_time(e["end"]) >= 0.0
    finally:
        c.close()
        dist.destroy_process_group()


def test_zipf_synthetic_vs_oracle(ctx):
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    n = 24 << 20
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_zipf(t.data_ptr(), n, 0x5EED2026, 0, 1 << 16, 1.1)
    host = t[:n].cpu().numpy().tobytes()
    ctx.job_begin(M.APP_WC, 64)
    ctx.set_input(t.data_ptr(), [0, n])
    ctx.map()
    ctx.reduce()
    got = ctx.outputs()
    exp = O.wc([host], 64, O.FAST)
    assert got == exp


@pytest.mark.parametrize("vocab,R", [(1 << 16, 64), (1 << 10, 7)])
def test_zipf_unicode_synthetic_vs_oracle(ctx, vocab, R):
    """Gutenberg-like Unicode Zipf text (mrg_gen_text style 1): wc and the indexer against the oracle."""
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import run_wc
    n = 12 << 20
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_text(t.data_ptr(), n, 0x5EED2026, 1, vocab, 1.1, 1)
    host = t[:n].cpu().numpy().tobytes()
    host.decode("utf-8")  # the generator writes valid UTF-8
    assert sum(1 for i in range(0, n, 1024) if max(host[i:i + 1024]) >= 0x80) > 0.9 * (n // 1024)
    ctx.job_begin(M.APP_WC, R)
    ctx.set_input(t.data_ptr(), [0, n])
    ctx.map()
    ctx.reduce()
    assert ctx.outputs() == O.wc([host], R, O.FAST)
    docs = [host[i * (n // 4):(i + 1) * (n // 4)] for i in range(4)]
    docs = [d[d.index(b" ") + 1:] if i else d for i, d in enumerate(docs)]  # whole codepoints per document
    docs = [d[:d.rindex(b" ")] for d in docs]
    names = [f"data/u-{i}.txt" for i in range(4)]
    assert run_wc(ctx, docs, R, app=M.APP_INDEXER, names=names) == O.indexer(docs, names, R)


def test_unique_synthetic_vs_oracle(ctx):
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    n = 8 << 20
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_unique(t.data_ptr(), n, 0xC5, 3)
    host = t[:n].cpu().numpy().tobytes()
    ctx.job_begin(M.APP_WC, 16)
    ctx.set_input(t.data_ptr(), [0, n])
    ctx.map()
    ctx.reduce()
    assert ctx.outputs() == O.wc([host], 16, O.FAST)


def test_run_job_cli_files(tmp_path, corpus):
    import mapreduce_rust_amd as M
    d = tmp_path / "data"
    d.mkdir()
    files = []
    for m in range(6):
        (d / f"gut-{m}.txt").write_bytes(corpus[m])
        files.append(f"data/gut-{m}.txt")
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        M.native.run_job(files, 10, M.APP_WC, ".")
    finally:
        os.chdir(cwd)
    for r in range(10):
        assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["wc"]["10"][f"mr-{r}.txt"]


def test_worker_tasks_through_files(tmp_path, corpus):
    """Reference task structure: 6 map tasks then 10 reduce tasks, hand-off through files."""
    from mapreduce_rust_amd.worker import Worker
    (tmp_path / "data").mkdir()
    for m in range(6):
        (tmp_path / "data" / f"gut-{m}.txt").write_bytes(corpus[m])
    w = Worker(6, 10, cwd=str(tmp_path), intermediates="records")
    for m in range(6):
        assert w.map(m)
    w2 = Worker(6, 10, cwd=str(tmp_path), intermediates="records")   # a second worker process would do the same
    for r in range(10):
        assert w2.reduce(r)
        assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["wc"]["10"][f"mr-{r}.txt"], r
    w.close()
    w2.close()


def test_worker_indexer_tasks(tmp_path, corpus):
    from mapreduce_rust_amd.worker import Worker
    (tmp_path / "data").mkdir()
    for m in range(6):
        (tmp_path / "data" / f"gut-{m}.txt").write_bytes(corpus[m])
    w = Worker(6, 10, app="indexer", cwd=str(tmp_path))
    for m in range(6):
        w.map(m)
    for r in range(10):
        w.reduce(r)
        assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["indexer"]["10"][f"mr-{r}.txt"], r
    w.close()


# ---- final.txt (src/run.sh:16-20, LC_ALL=C) built on the device: SURVEY.md §8 row f3

def _final_of(outs):
    """run.sh:16-20 restated: every line of every mr-{r}.txt, sorted bytewise."""
    lines = [l for o in outs for l in o.split(b"\n") if l]
    return b"".join(l + b"\n" for l in sorted(lines))


@pytest.mark.parametrize("R", ["10", "1", "3", "64"])
def test_final_txt_golden(ctx, corpus, R):
    from gpu_util import run_wc
    outs = run_wc(ctx, corpus, int(R))
    fin = ctx.final()
    assert sha(fin) == GOLDEN["wc"][R]["final.txt"]
    assert fin == _final_of(outs)


def test_final_txt_no_drop_and_collisions(ctx, corpus):
    """Last groups kept (nothing dropped) and forced internal hash collisions (long-key tie-breaks)."""
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    for flags in (M.FLAG_NO_COMPAT_DROP_LAST, M.debug_hash_bits(4), M.FLAG_NO_COMPAT_DROP_LAST | M.debug_hash_bits(1)):
        outs = run_wc(ctx, corpus[:3], 7, flags=flags)
        assert ctx.final() == _final_of(outs), flags


def test_final_txt_long_keys_and_unicode(ctx):
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    rnd = random.Random(7)
    words = ["x" * n + s for n in (15, 16, 17, 30) for s in ("", "a", "b", "é")] + ["naïve", "ſong", "Ærø", "a"]
    text = " ".join(rnd.choice(words) for _ in range(5000)).encode()
    for flags in (0, M.FLAG_NO_COMPAT_DROP_LAST):
        outs = run_wc(ctx, [text], 5, flags=flags)
        assert ctx.final() == _final_of(outs)


def test_final_txt_indexer(ctx, corpus):
    import mapreduce_rust_amd as M
    from gpu_util import run_wc
    names = [f"data/gut-{m}.txt" for m in range(6)]
    outs = run_wc(ctx, corpus, 10, app=M.APP_INDEXER, names=names)
    assert ctx.final() == _final_of(outs)


def test_final_txt_empty(ctx):
    from gpu_util import run_wc
    run_wc(ctx, [b"", b"  \n"], 4)
    assert ctx.final() == b""


def test_run_job_writes_final_txt(tmp_path, corpus):
    import mapreduce_rust_amd as M
    d = tmp_path / "data"
    d.mkdir()
    files = []
    for m in range(6):
        (d / f"gut-{m}.txt").write_bytes(corpus[m])
        files.append(f"data/gut-{m}.txt")
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        M.native.run_job(files, 10, M.APP_WC, ".", M.FLAG_FINAL_TXT)
    finally:
        os.chdir(cwd)
    assert sha((tmp_path / "final.txt").read_bytes()) == GOLDEN["wc"]["10"]["final.txt"]


# ---- wide (sort-based) aggregation: the high-cardinality path (C5) forced on small inputs

@pytest.fixture
def wide():
    os.environ["MRG_WIDE"] = "1"
    yield
    del os.environ["MRG_WIDE"]


@pytest.mark.parametrize("R", ["10", "64"])
def test_wide_path_c1_golden(ctx, corpus, wide, R):
    from gpu_util import run_wc
    outs = run_wc(ctx, corpus, int(R))
    g = GOLDEN["wc"][R]
    assert [sha(o) for o in outs] == [g[f"mr-{r}.txt"] for r in range(int(R))]
    assert sha(ctx.final()) == g["final.txt"]


def test_wide_path_synthetic_and_unicode(ctx, wide):
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import run_wc
    n = 8 << 20
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda:0")
    ctx.gen_unique(t.data_ptr(), n, 0xC5, 5)
    host = t[:n].cpu().numpy().tobytes()
    ctx.job_begin(M.APP_WC, 16)
    ctx.set_input(t.data_ptr(), [0, n])
    ctx.map()
    ctx.reduce()
    assert ctx.outputs() == O.wc([host], 16, O.FAST)
    ctx.gen_zipf(t.data_ptr(), n, 0x5EED2026, 1, 1 << 14, 1.1)
    host = t[:n].cpu().numpy().tobytes()
    ctx.job_begin(M.APP_WC, 7)
    ctx.set_input(t.data_ptr(), [0, n])
    ctx.map()
    ctx.reduce()
    assert ctx.outputs() == O.wc([host], 7, O.FAST)
    rnd = random.Random(11)
    words = ["x" * k + e for k in (3, 16, 17, 40) for e in ("", "é", "q")] + ["naïve", "a", "don't"]
    text = " ".join(rnd.choice(words) for _ in range(20000)).encode()
    for flags in (0, M.debug_hash_bits(3)):
        assert run_wc(ctx, [text], 5, flags=flags) == O.wc([text], 5, O.FAST), flags


# ---- the reference's text intermediates mr-{m}-{r}.txt

from reduce_twin import REDUCE_EDGE_CASES, ref_reduce as _ref_reduce  # noqa: E402


@pytest.mark.parametrize("R", ["10", "1", "3", "64"])
def test_map_text_golden_intermediates(ctx, corpus, R):
    n = int(R)
    blobs = []
    for m in range(6):
        blobs += ctx.map_text(corpus[m], n)
    assert sha(b"".join(blobs)) == GOLDEN["wc"][R]["intermediates"]
    outs = [ctx.reduce_text([blobs[m * n + r] for m in range(6)]) for r in range(n)]
    assert [sha(o) for o in outs] == [GOLDEN["wc"][R][f"mr-{r}.txt"] for r in range(n)]


def test_map_text_unicode_and_long_tokens(ctx):
    import oracle_lib as O
    rnd = random.Random(5)
    words = ["x" * k + e for k in (3, 16, 17, 40) for e in ("", "é", "q")] + ["naïve", "a", "don't", "--", "ſong",
                                                                              "«quoted»", "1685-1732"]
    seps = [" ", "\n", "\t", "　", "   "]
    text = "".join(rnd.choice(words) + rnd.choice(seps) for _ in range(30000)).encode()
    for n in (1, 7):
        parts = ctx.map_text(text, n)
        assert [ctx.reduce_text([p]) for p in parts] == [_ref_reduce([p]) for p in parts]
        assert [ctx.reduce_text([p]) for p in parts] == O.wc([text], n, O.FAST)


def test_reduce_text_edge_cases(ctx):
    import mapreduce_rust_amd as M
    cases = REDUCE_EDGE_CASES
    for files in cases:
        for flags, drop in ((0, True), (M.FLAG_NO_COMPAT_DROP_LAST, False)):
            assert ctx.reduce_text(files, flags) == _ref_reduce(files, drop), (files, flags)


def test_reduce_text_errors(ctx):
    import mapreduce_rust_amd as M
    for files, code in (([b"a b c\n"], M.native.EINVAL), ([b"abc\n"], M.native.EINVAL),
                        ([b"a 1\n", b"\xff 1\n"], M.native.EUTF8), ([b"a\x00b 1\n"], M.native.EINVAL)):
        with pytest.raises(M.MrgError) as ei:
            ctx.reduce_text(files)
        assert ei.value.code == code, files
    with pytest.raises(M.MrgError) as ei:
        ctx.map_text(b"ok \xe2\x82 bad", 4)
    assert ei.value.code == M.native.EUTF8


def test_worker_text_intermediates_through_files(tmp_path, corpus):
    """Reference task structure with the reference's own intermediate files (default for wc)."""
    from mapreduce_rust_amd.worker import Worker
    (tmp_path / "data").mkdir()
    for m in range(6):
        (tmp_path / "data" / f"gut-{m}.txt").write_bytes(corpus[m])
    w = Worker(6, 10, cwd=str(tmp_path))
    for m in range(6):
        assert w.map(m)
    inter = b"".join((tmp_path / f"mr-{m}-{r}.txt").read_bytes() for m in range(6) for r in range(10))
    assert sha(inter) == GOLDEN["wc"]["10"]["intermediates"]
    for r in range(10):
        assert w.reduce(r)
        assert sha((tmp_path / f"mr-{r}.txt").read_bytes()) == GOLDEN["wc"]["10"][f"mr-{r}.txt"], r
    w.close()


@pytest.mark.parametrize("G", [1, 3, 300])
def test_export_import_many_owners(ctx, corpus, G):
    """The export by owner (part % G) and the re-import, at 1, 3 and 300 owners (300: more owners
    than the export kernels count in LDS, so the per-key device-atomic path runs), with long (> 16
    byte) keys in the exchange heap: the union of the owners' partitions equals the oracle."""
    import torch
    import mapreduce_rust_amd as M
    import oracle_lib as O
    from gpu_util import to_device
    R = 600
    longs = (b"pneumonoultramicroscopicsilicovolcanoconiosis supercalifragilisticexpialidocious "
             b"antidisestablishmentarianism floccinaucinihilipilification ") * 50
    docs = [corpus[0], corpus[1] + b" " + longs, corpus[2], longs + corpus[3]]
    shards = [docs[0:2], docs[2:4]]
    sends = []
    for sh in shards:
        t, off = to_device(sh)
        ctx.job_begin(M.APP_WC, R)
        ctx.set_input(t.data_ptr(), off)
        ctx.map()
        rec, heap = ctx.export_sizes(G)
        drec = torch.empty(max(sum(rec), 1) * X, dtype=torch.uint8, device="cuda:0")
        dheap = torch.empty(max(sum(heap), 1), dtype=torch.uint8, device="cuda:0")
        ctx.export(drec.data_ptr(), dheap.data_ptr())
        sends.append((drec.cpu(), dheap.cpu(), rec, heap))
    exp = O.wc(docs, R, O.FAST)
    got = [None] * R
    for owner in range(G):
        recs, heaps, sr, shp = [], [], [], []
        for drec, dheap, rec, heap in sends:
            ro = sum(rec[:owner]) * X
            ho = sum(heap[:owner])
            recs.append(drec[ro:ro + rec[owner] * X])
            heaps.append(dheap[ho:ho + heap[owner]])
            sr.append(rec[owner])
            shp.append(heap[owner])
        Rt = torch.cat(recs + [torch.zeros(X, dtype=torch.uint8)]).to("cuda:0")
        Ht = torch.cat(heaps + [torch.zeros(1, dtype=torch.uint8)]).to("cuda:0")
        ctx.job_begin(M.APP_WC, R)
        ctx.import_(Rt.data_ptr(), sum(sr), Ht.data_ptr(), sum(shp), sr, shp)
        ctx.reduce()
        o = ctx.outputs()
        for r in range(R):
            if r % G == owner:
                got[r] = o[r]
            else:
                assert o[r] == b"", (owner, r)
    assert got == exp
