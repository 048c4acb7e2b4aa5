#!/usr/bin/env python3
"""GPU debugging aid: full mr-0.txt (R = 1) of a fixed small multi-document input, with and without
the last-group drop, beside the oracle's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mapreduce_rust_amd as M  # noqa: E402
import oracle_lib as O  # noqa: E402
from gpu_util import run_wc  # noqa: E402

ctx = M.Context(0)
cases = [
    [b'X\na\taZad_  X_\xe2\x80\xa8b\xd0\xb6\xd0\xb6\xc3\x9fZ  ZXb ', b'\xc3\xa9  '],
    [b'X\na\taZad_  X_\xe2\x80\xa8b\xd0\xb6\xd0\xb6\xc3\x9fZ  ZXb '],
    [b'\xc3\xa9  '],
    [b'0123456789abcdefghijklmnopqrstu ', b'\xc3\xa9  '],
    [b'X\na\taZad_  X_   b\xd0\xb6\xd0\xb6\xc3\x9fZ  ZXb ', b'\xc3\xa9  '],
]
for docs in cases:
    for flags in (0, M.FLAG_NO_COMPAT_DROP_LAST):
        got = run_wc(ctx, docs, 1, flags=flags)[0]
        print(f"docs {[len(d) for d in docs]} flags {flags} tokens {ctx.stats()['tokens']} nonascii {ctx.stats()['nonascii_tiles']}")
        print("   gpu   ", got)
    print("   oracle", O.wc(docs, 1, O.FAST)[0], flush=True)
ctx.close()
