"""r06 cold-job probe: C3 input (40 x 256 MiB Zipf) resident; context A runs 3 jobs, is closed, context B
(whose pool starts from A's cached device blocks) runs 2 jobs; per job the HIP-event stage times, the
pool's hipMalloc count/ms and the wall time.  Tells first-touch of fresh memory from first-job logic."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import mapreduce_rust_amd as M

nf, fb = 40, 256 << 20
g = M.Context(0)
buf = torch.empty(nf * fb + 64, dtype=torch.uint8, device="cuda:0")
for i in range(nf):
    g.gen_zipf(buf.data_ptr() + i * fb, fb, 0x5EED2026, i, 1 << 20, 1.1)
torch.cuda.synchronize()
off = [i * fb for i in range(nf + 1)]


def jobs(tag, n, idle=0.0):
    c = M.Context(0)
    c.set_timing(True)
    for j in range(n):
        if idle:
            time.sleep(idle)   # the GPU idles (as through mrg_run_job's file read)
        a0 = c.pool_alloc_stats()
        torch.cuda.synchronize()
        t = time.perf_counter()
        c.job_begin(M.APP_WC, 64)
        c.set_input(buf.data_ptr(), off)
        c.map()
        c.reduce()
        torch.cuda.synchronize()
        w = (time.perf_counter() - t) * 1e3
        a1 = c.pool_alloc_stats()
        s = c.stats()
        print(f"{tag} job {j}: wall {w:.2f} ms, map {s['ms_map']:.3f} agg {s['ms_aggregate']:.3f} sort {s['ms_sort']:.3f} "
              f"fmt {s['ms_format']:.3f}, launches {s['map_launches']}, spec {s['spec_agg']}, "
              f"hipMalloc {a1[0] - a0[0]} ({(a1[1] - a0[1]) / 2**30:.2f} GiB, {a1[2] - a0[2]:.2f} ms)", flush=True)
    c.close()


if os.environ.get("PROBE_DONLY"):
    jobs("A", 1)
else:
    jobs("A", 3)
    jobs("B", 2)
# D: the same bytes copied back in by DMA (as mrg_run_job's read path does) into the same buffer
host = torch.empty(nf * fb, dtype=torch.uint8, pin_memory=True)
host.copy_(buf[:nf * fb])
torch.cuda.synchronize()
buf[:nf * fb].copy_(host, non_blocking=True)
torch.cuda.synchronize()
jobs("D (input just DMA-written)", 3)
jobs("E (no rewrite, 0.3 s idle before each job)", 3, idle=0.3)
if os.environ.get("PROBE_DONLY"):
    sys.exit(0)
os.environ["MRG_WIDE_MAP"] = "0"      # no cold-context sample
jobs("C (no sample)", 2)
del os.environ["MRG_WIDE_MAP"]
t = time.perf_counter()
st = M.native.run_job([], 64, M.APP_WC, "/tmp") if False else None
