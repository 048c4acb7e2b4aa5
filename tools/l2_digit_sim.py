import numpy as np, sys
NB = int(sys.argv[1]) if len(sys.argv) > 1 else 3   # digit bytes
rng = np.random.default_rng(5)
alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
def keys(n):
    K = alpha[rng.integers(0, 36, size=(n, 12))]
    return np.sort(K.view('S12').ravel())
allk = keys(2_000_000)
def kb(k, j): return k[j] if j < len(k) else 0
bad = 0; sizes = []; used = []
for trial in range(60):
    i = rng.integers(0, len(allk) - 300000); j = i + rng.integers(200, 300000)
    lo, hi = allk[i], allk[j]
    ks = allk[i:j]
    nb = len(ks)
    S = min(nb, 2048)
    smp = [ks[((2 * k + 1) * nb) // (2 * S)] for k in range(S)]
    f = smp[0]
    P = 0
    for pos in range(16):
        if any(kb(s, pos) != kb(f, pos) for s in smp) or kb(lo, pos) != kb(hi, pos):
            P = pos; break
    tabs = []; nv = []
    for t in range(NB):
        pres = np.zeros(256, np.int64)
        for s in smp: pres[kb(s, P + t)] = 1
        excl = np.cumsum(pres) - pres
        tabs.append((excl, pres)); nv.append(int(pres.sum()))
    Rs = [v + 1 for v in nv]
    N = 1
    for r_ in Rs: N *= r_
    M = (8192 << 32) // N if N > 8192 else (1 << 32)
    def dig(k):
        x = 0; live = 1
        for t in range(NB):
            b = kb(k, P + t)
            c = int(tabs[t][0][b]) if live else 0
            live = live and int(tabs[t][1][b])
            x = x * Rs[t] + c
        return (x * M) >> 32
    d = [dig(k) for k in ks]
    if any(d[x] > d[x + 1] for x in range(len(d) - 1)):
        bad += 1
        x = next(x for x in range(len(d) - 1) if d[x] > d[x + 1])
        print("non-monotone", trial, P, ks[x], ks[x + 1], d[x], d[x + 1], nv)
        if bad > 3: break
    if nb > 100000: sizes.append(np.bincount(d).max()); used.append((np.bincount(d) > 0).sum())
print("bytes", NB, "bad", bad, "max digit bucket (nb>100k) mean", np.mean(sizes), "digits used", np.mean(used))
