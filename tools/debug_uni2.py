#!/usr/bin/env python3
"""GPU debugging aid: the random-Unicode parity case (tests/test_gpu_parity.py) repeated on one
context, R = 1 and 7, full output bytes against the oracle; reports which repetitions differ and how."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mapreduce_rust_amd as M  # noqa: E402
import oracle_lib as O  # noqa: E402
import test_gpu_parity as T  # noqa: E402
from gpu_util import run_wc  # noqa: E402

ctx = M.Context(0)
for seed in [int(a) for a in sys.argv[1:]] or [3]:
    rng = random.Random(seed)
    docs = [T._rand_text(rng, rng.randint(0, 3000), T.ALPHA[: 6 + seed * 3], T.SEPS, max_len=[5, 12, 40][seed % 3])
            for _ in range(rng.randint(1, 5))]
    for rep in range(4):
        for R in (1, 7):
            got = run_wc(ctx, docs, R)
            exp = O.wc(docs, R, O.FAST)
            st = ctx.stats()
            if got != exp:
                for r in range(R):
                    if got[r] != exp[r]:
                        gl, el = got[r].split(b"\n"), exp[r].split(b"\n")
                        d = [(i, a, b) for i, (a, b) in enumerate(zip(gl, el)) if a != b][:3]
                        print(f"seed {seed} rep {rep} R {R} part {r}: {len(gl)} vs {len(el)} lines; first diffs {d}")
                        break
                print("   stats", {k: st[k] for k in ("tokens", "map_records", "distinct_keys", "spec_agg", "agg_path",
                                                      "nonascii_tiles", "map_launches", "agg_launches")}, flush=True)
            else:
                print(f"seed {seed} rep {rep} R {R}: ok (spec_agg {st['spec_agg']})", flush=True)
ctx.close()
