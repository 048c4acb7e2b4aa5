"""Debug: C5 slice output of the library at MRG_LIB, written to /tmp/ww_<tag>.bin (on the box), or with
--cmp A B: the byte differences of two such dumps (count, first positions with context)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if sys.argv[1] == "--cmp":
    import numpy as np
    a = np.fromfile(sys.argv[2], dtype=np.uint8)
    b = np.fromfile(sys.argv[3], dtype=np.uint8)
    print("sizes", a.size, b.size)
    n = min(a.size, b.size)
    d = np.nonzero(a[:n] != b[:n])[0]
    print("differing bytes", d.size)
    for p in d[:6]:
        lo = max(0, p - 40)
        print(p, bytes(a[lo:p + 24]), "|", bytes(b[lo:p + 24]))
    if d.size:
        nl = np.nonzero(a == 10)[0]
        li = np.searchsorted(nl, d)          # line index of each differing byte
        ls = np.where(li > 0, nl[np.maximum(li - 1, 0)] + 1, 0)
        col = d - ls
        x = a[d] ^ b[d]
        print("column histogram", np.bincount(col)[:20].tolist())
        print("xor values", np.unique(x, return_counts=True))
        print("first 80 line indices", li[:80].tolist())
        print("line index mod 64 histogram", np.bincount(li % 64, minlength=64).tolist())
        print("pos mod 16 histogram", np.bincount(d % 16, minlength=16).tolist())
        # lines with a count other than 1 within +-64 lines of the first corrupted lines of each run
        runs = [li[0]] + [li[i] for i in range(1, min(li.size, 20000)) if li[i] - li[i - 1] > 8]
        for r0 in runs[:8]:
            lo = nl[max(r0 - 70, 0)] + 1
            hi = nl[min(r0 + 70, nl.size - 1)]
            txt = bytes(a[lo:hi]).split(b"\n")
            odd = [t for t in txt if not t.endswith(b" 1")]
            print("run at line", int(r0), "non-1 counts nearby:", odd[:6])
    sys.exit(0)
import torch
import mapreduce_rust_amd as M
tag = sys.argv[1]
nf, fb = 4, 256 << 20
ctx = M.Context(0)
buf = torch.empty(nf * fb + 64, dtype=torch.uint8, device="cuda:0")
for i in range(nf):
    ctx.gen_unique(buf.data_ptr() + i * fb, fb, 0xC5C5, i)
torch.cuda.synchronize()
ctx.job_begin(M.APP_WC, 64)
ctx.set_input(buf.data_ptr(), [i * fb for i in range(nf + 1)])
ctx.map()
n = ctx.reduce()
outs = ctx.outputs()
with open(f"/tmp/ww_{tag}.bin", "wb") as f:
    for o in outs:
        f.write(o)
print(tag, "bytes", n, ctx.stats()["distinct_keys"])
