import numpy as np
rng = np.random.default_rng(5)
alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
def keys(n):
    K = alpha[rng.integers(0, 36, size=(n, 12))]
    return np.sort(K.view('S12').ravel())
allk = keys(2_000_000)
def kb(k, j): return k[j] if j < len(k) else 0
bad = 0; sizes = []
for trial in range(400):
    i = rng.integers(0, len(allk) - 30000); j = i + rng.integers(200, 30000)
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
    for t in range(3):
        pres = np.zeros(256, np.int64)
        for s in smp: pres[kb(s, P + t)] = 1
        excl = np.cumsum(pres) - pres
        tabs.append((excl, pres)); nv.append(int(pres.sum()))
    R1, R2 = nv[1] + 1, nv[2] + 1
    N = (nv[0] + 1) * R1 * R2
    M = (8192 << 32) // N if N > 8192 else (1 << 32)
    def dig(k):
        b0, b1, b2 = kb(k, P), kb(k, P + 1), kb(k, P + 2)
        c0, p0 = int(tabs[0][0][b0]), int(tabs[0][1][b0])
        c1 = int(tabs[1][0][b1]) if p0 else 0; p1 = p0 and int(tabs[1][1][b1])
        c2 = int(tabs[2][0][b2]) if p1 else 0
        return (((c0 * R1 + c1) * R2 + c2) * M) >> 32
    d = [dig(k) for k in ks]
    if any(d[x] > d[x + 1] for x in range(len(d) - 1)):
        bad += 1
        x = next(x for x in range(len(d) - 1) if d[x] > d[x + 1])
        print("non-monotone", trial, P, ks[x], ks[x + 1], d[x], d[x + 1], nv)
        if bad > 3: break
    if nb > 10000: sizes.append(np.bincount(d).max())
print("bad", bad, "max digit bucket (nb>10k) mean", np.mean(sizes))
