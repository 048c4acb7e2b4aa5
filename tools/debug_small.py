#!/usr/bin/env python3
"""GPU debugging aid: run small word-count inputs through the C ABI and print the first
differences against the C oracle (R = 1, no drop-last), plus the token counts."""
import collections
import gzip
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mapreduce_rust_amd as M  # noqa: E402
import oracle_lib as O  # noqa: E402
from gpu_util import run_wc  # noqa: E402


def parse(b):
    d = collections.Counter()
    for line in b.decode().splitlines():
        k, v = line.rsplit(" ", 1)
        d[k] += int(v)
    return d


def check(ctx, name, docs):
    flags = M.FLAG_NO_COMPAT_DROP_LAST if hasattr(M, "FLAG_NO_COMPAT_DROP_LAST") else 0
    got = run_wc(ctx, docs, 1, flags=flags)[0]
    exp = None
    st = ctx.stats()
    toks = sum(len(O.tokens(d)) for d in docs)
    g = parse(got)
    if exp is None:
        e = collections.Counter()
        for d in docs:
            e.update(t.decode() for t in O.tokens(d) if t)
    else:
        e = parse(exp)
    diff = [(k, g.get(k, 0), e.get(k, 0)) for k in set(g) | set(e) if g.get(k, 0) != e.get(k, 0)]
    print(f"{name}: gpu tokens {st['tokens']} oracle tokens {toks}; keys gpu {len(g)} oracle {len(e)}; "
          f"{len(diff)} differing keys", flush=True)
    for k, a, b in sorted(diff, key=lambda x: -abs(x[1] - x[2]))[:12]:
        print(f"    {k!r}: gpu {a} oracle {b}")


def main():
    ctx = M.Context(0)
    unit = b"five six seven "
    check(ctx, "l0=4 n=100", [b"ab a", unit * 100])
    check(ctx, "l0=4 n=100 distinct", [b"ab a", b"".join(b"w%03da w%03db w%03dc " % (i, i, i) for i in range(60))])
    check(ctx, "l0=5700 n=1", [(b"ab " * 2000)[:5700], unit])
    check(ctx, "l0=5700 distinct", [b"".join(b"x%04d " % i for i in range(950))[:5700], unit])
    ctx.close()


if __name__ == "__main__":
    main()
