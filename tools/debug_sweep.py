#!/usr/bin/env python3
"""GPU debugging aid: sweep input sizes/offsets, report which inputs give extra/missing tokens."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mapreduce_rust_amd as M  # noqa: E402
import oracle_lib as O  # noqa: E402
from gpu_util import run_wc  # noqa: E402


def main():
    ctx = M.Context(0)
    unit = b"five six seven "
    for pad in (0, 1, 5):
        for n in (1, 60, 68, 69, 70, 130, 137, 138, 140, 200, 273, 274, 300):
            doc = b"x" * pad + b" " + unit * n
            run_wc(ctx, [doc], 1, flags=M.FLAG_NO_COMPAT_DROP_LAST)
            st = ctx.stats()
            exp = len([t for t in O.tokens(doc) if t])
            if st["tokens"] != exp:
                print(f"pad {pad} n {n} len {len(doc)}: gpu {st['tokens']} oracle {exp}", flush=True)
    for l0 in (1, 2, 4, 7, 15, 16, 17, 100, 1000, 2040, 2047, 2048, 2049, 5700):
        for n in (1, 20, 100, 200):
            d0 = (b"ab " * 2000)[:l0]
            d1 = unit * n
            run_wc(ctx, [d0, d1], 1, flags=M.FLAG_NO_COMPAT_DROP_LAST)
            st = ctx.stats()
            exp = len([t for t in O.tokens(d0) if t]) + len([t for t in O.tokens(d1) if t])
            if st["tokens"] != exp:
                print(f"2docs l0 {l0} n {n}: gpu {st['tokens']} oracle {exp}", flush=True)
    print("sweep done", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
