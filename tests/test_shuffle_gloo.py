"""CPU test of the multi-GPU shuffle path (mapreduce_rust_amd.shuffle) with the gloo backend.

World size 2 (and 3).  Each rank plays the part of one GPU: it tokenizes its shard of the bundled
corpus with the oracle (test infrastructure), packs its per-key counts into exchange records exactly
as mrg_job_export lays them out (include/mrgpu.h: 24-byte records ordered by owner r % G, short keys
packed in the record, long keys in a heap addressed per sender segment), runs the real alltoall_exchange, unpacks what it received
the way mrg_job_import does, and reduces the partitions it owns.  The union of all ranks' outputs
must equal the single-process oracle job byte for byte (golden digests of SURVEY.md §8(c)).
"""
import gzip
import hashlib
import json
import os
import struct
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _corpus():
    return [gzip.open(os.path.join(HERE, "golden", "corpus", f"gut-{m}.txt.gz")).read() for m in range(6)]


def pack(counts, n_reduce, n_owners, key_hash):
    """Per-key counts -> (records, heap, rec_counts, heap_counts), records grouped by owner."""
    by_owner = [[] for _ in range(n_owners)]
    for k, c in counts.items():
        r = key_hash(k) % n_reduce
        by_owner[r % n_owners].append((k, c))
    recs, heap = bytearray(), bytearray()
    rc, hc = [], []
    for o in range(n_owners):
        seg = bytearray()
        n = 0
        for k, c in by_owner[o]:
            if len(k) > 16:  # long form: heap offset, 64-bit count
                recs += struct.pack("<QQII", len(seg), c, 0xFFFFFFFF, len(k))
                seg += k
                n += 1
                continue
            pre = k.ljust(16, b"\0")
            k0 = int.from_bytes(pre[:8], "big")
            k1 = int.from_bytes(pre[8:], "big")
            while True:  # short form: the count in 32 bits, larger counts over several records
                part = min(c, 0xFFFFFFFF)
                recs += struct.pack("<QQII", k0, k1, part, len(k))
                n += 1
                c -= part
                if c == 0:
                    break
        rc.append(n)
        hc.append(len(seg))
        heap += seg
    return bytes(recs), bytes(heap), rc, hc


def unpack(recv_rec, recv_heap, r_rec, r_heap):
    """mrg_job_import semantics: sum counts per key across senders."""
    out = {}
    hbase = 0
    i = 0
    for n, hb in zip(r_rec, r_heap):
        for _ in range(n):
            a, b, v, ln = struct.unpack_from("<QQII", recv_rec, i * 24)
            if ln > 16:
                k = bytes(recv_heap[hbase + a:hbase + a + ln])
                c = b
            else:
                k = (a.to_bytes(8, "big") + b.to_bytes(8, "big"))[:ln]
                c = v
            out[k] = out.get(k, 0) + c
            i += 1
        hbase += hb
    return out


def reduce_owned(counts, n_reduce, rank, world, key_hash):
    parts = {r: [] for r in range(n_reduce) if r % world == rank}
    for k, c in counts.items():
        r = key_hash(k) % n_reduce
        assert r in parts, "received a key of a partition this rank does not own"
        parts[r].append((k, c))
    outs = {}
    for r, kv in parts.items():
        kv.sort()
        outs[r] = b"".join(k + b" " + str(c).encode() + b"\n" for k, c in kv[:-1])  # last group dropped
    return outs


def _worker(rank, world, init_file, n_reduce, result_dir):
    import sys
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.dirname(HERE))
    import oracle_lib as O
    from mapreduce_rust_amd import shuffle as S
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    files = _corpus()
    counts = {}
    for m in S.shard_files(len(files), rank, world):
        for t in O.tokens(files[m]):
            counts[t] = counts.get(t, 0) + 1
    rec, heap, rc, hc = pack(counts, n_reduce, world, O.key_hash)
    send_rec = torch.frombuffer(bytearray(rec) + bytearray(1), dtype=torch.uint8)
    send_heap = torch.frombuffer(bytearray(heap) + bytearray(1), dtype=torch.uint8)
    recv_rec, recv_heap, r_rec, r_heap = S.alltoall_exchange(send_rec, send_heap, rc, hc)
    got = unpack(recv_rec.numpy().tobytes(), recv_heap.numpy().tobytes(), r_rec, r_heap)
    outs = reduce_owned(got, n_reduce, rank, world, O.key_hash)
    with open(os.path.join(result_dir, f"rank{rank}.json"), "w") as f:
        json.dump({str(r): hashlib.sha256(b).hexdigest() for r, b in outs.items()}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shuffle_gloo_matches_golden(world):
    golden = json.load(open(os.path.join(HERE, "golden", "golden.json")))
    with tempfile.TemporaryDirectory() as d:
        init = os.path.join(d, "init")
        mp.spawn(_worker, args=(world, init, 10, d), nprocs=world, join=True)
        merged = {}
        for rk in range(world):
            merged.update(json.load(open(os.path.join(d, f"rank{rk}.json"))))
    assert sorted(int(r) for r in merged) == list(range(10))
    for r in range(10):
        assert merged[str(r)] == golden["wc"]["10"][f"mr-{r}.txt"], r


def test_owner_plan():
    from mapreduce_rust_amd import shuffle as S
    assert [S.owner_of(r, 8) for r in range(10)] == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]
    assert S.shard_files(10, 1, 4) == [1, 5, 9]
    # every file mapped exactly once over the ranks
    got = sorted(m for g in range(3) for m in S.shard_files(7, g, 3))
    assert got == list(range(7))
