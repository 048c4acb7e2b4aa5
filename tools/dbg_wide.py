"""Debug helper: a small near-unique job through the wide path vs the oracle; prints the first
differing lines of each partition that differs."""
import os, sys
_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [_R, os.path.join(_R, "tests")]
import test_gpu_scale as T
import mapreduce_rust_amd as M
import oracle_lib as O

nf, fb = int(sys.argv[1]) if len(sys.argv) > 1 else 1, (int(sys.argv[2]) if len(sys.argv) > 2 else 64) * T.MIB
ctx = M.Context(0)
buf = T._generate(ctx, "unique", nf, fb, 0xC5C5)
got = T._run_job(ctx, buf, nf, fb, 64)
print("stats", ctx.stats(), flush=True)
files = T._host_files(buf, nf, fb)
exp = O.wc_mt(files, 64, threads=16)
nbad = 0
for r in range(64):
    if got[r] == exp[r]:
        continue
    nbad += 1
    g, e = got[r].split(b"\n"), exp[r].split(b"\n")
    print(f"part {r}: got {len(g)} lines, exp {len(e)}")
    for i in range(min(len(g), len(e))):
        if g[i] != e[i]:
            print("  first diff at line", i)
            for k in range(max(0, i - 3), min(i + 4, len(g), len(e))):
                print("   ", k, g[k], e[k])
            break
    if nbad >= 4:
        break
print("bad partitions:", nbad)
