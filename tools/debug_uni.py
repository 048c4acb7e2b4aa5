#!/usr/bin/env python3
"""GPU debugging aid for the non-ASCII tile path: the random-Unicode parity case of
tests/test_gpu_parity.py (seed from argv), its differing keys against the oracle, then a greedy
shrink of the failing document (drop token/separator pairs while the GPU still differs)."""
import collections
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import mapreduce_rust_amd as M  # noqa: E402
import oracle_lib as O  # noqa: E402
from gpu_util import run_wc  # noqa: E402

from test_gpu_parity import ALPHA, SEPS  # noqa: E402
F = M.FLAG_NO_COMPAT_DROP_LAST


def pairs(rng, n, alphabet, seps, max_len):
    out = []
    for _ in range(n):
        L = rng.randint(1, max_len)
        out.append(("".join(rng.choice(alphabet) for _ in range(L)), rng.choice(seps)))
    return out


def enc(ps):
    return "".join(t + s for t, s in ps).encode()


def diff(ctx, docs, flags=0):
    """Keys whose counts differ between the GPU's mr-0.txt (R = 1) and the oracle's."""
    def parse(b):
        g = collections.Counter()
        for line in b.split(b"\n"):
            if line:
                k, v = line.rsplit(b" ", 1)
                g[k] += int(v)
        return g
    g = parse(run_wc(ctx, docs, 1, flags=flags)[0])
    e = parse(O.wc(docs, 1, O.FAST)[0] if not flags else b"".join(
        k + b" " + str(v).encode() + b"\n" for k, v in collections.Counter(
            t for d in docs for t in O.tokens(d) if t).items()))
    return [(k, g.get(k, 0), e.get(k, 0)) for k in set(g) | set(e) if g.get(k, 0) != e.get(k, 0)]


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ctx = M.Context(0)
    rng = random.Random(seed)
    docs_p = [pairs(rng, rng.randint(0, 3000), ALPHA[: 6 + seed * 3], SEPS, [5, 12, 40][seed % 3])
              for _ in range(rng.randint(1, 5))]
    docs = [enc(p) for p in docs_p]
    d = diff(ctx, docs)
    print(f"seed {seed}: {len(docs)} docs, {len(d)} differing keys", flush=True)
    for k, a, b in d[:20]:
        print(f"   {k!r} gpu {a} oracle {b}")
    # shrink every document (drop token/separator pairs) while the set of documents still differs
    cur = [list(p) for p in docs_p]
    for di in range(len(cur)):
        step = max(1, len(cur[di]) // 2)
        while step >= 1:
            j = 0
            while j < len(cur[di]):
                trial = [c if k != di else c[:j] + c[j + step:] for k, c in enumerate(cur)]
                if diff(ctx, [enc(c) for c in trial]):
                    cur = trial
                else:
                    j += step
            step //= 2
    bs = [enc(c) for c in cur]
    print(f"minimal: {[len(b) for b in bs]} bytes")
    for b in bs:
        print(f"   doc {b!r}")
    for k, a, bb in diff(ctx, bs):
        print(f"   {k!r} gpu {a} oracle {bb}")
    ctx.close()


if __name__ == "__main__":
    main()
