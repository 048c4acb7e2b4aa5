"""Device footprint of one C5 job on a fresh context: hipMalloc bytes of the pool (mrg_pool_alloc_stats),
for the sampled (MRG_WIDE_L2_SAMPLED=1) and the exact (default) wide-map L2, on FILES x 256 MiB of near-unique keys.
MRG_POOL_KEEP_GIB=0 so no context inherits another's blocks."""
import os, sys
os.environ["MRG_POOL_KEEP_GIB"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mapreduce_rust_amd as M

files = int(os.environ.get("FILES", "16"))
fb = 256 << 20
buf = torch.empty(files * fb + 64, dtype=torch.uint8, device="cuda:0")
with M.Context(0) as g:
    for i in range(files):
        g.gen_unique(buf.data_ptr() + i * fb, fb, 0xC5, i)
torch.cuda.synchronize()
doc_off = [i * fb for i in range(files + 1)]
for sampled in ("1", "0", "1", "0"):
    os.environ["MRG_WIDE_L2_SAMPLED"] = sampled
    with M.Context(0) as c:
        for rep in range(2):
            c.job_begin(M.APP_WC, 64)
            c.set_input(buf.data_ptr(), doc_off)
            c.map()
            c.reduce()
            n, b, ms = c.pool_alloc_stats()
            st = c.stats()
            print(f"L2_SAMPLED={sampled} job {rep}: {n} hipMalloc, {b / 2**30:.2f} GiB, {ms:.1f} ms; map_kind {st['map_kind']} keys {st['distinct_keys']}", flush=True)
