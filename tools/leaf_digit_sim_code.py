import os
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'leaf_digit_sim.py')).read().split("L = 256")[0])
L = 256
def scheme_code(a0, a1):
    f0, f1 = a0[0], a1[0]
    o0 = np.bitwise_or.reduce(a0 ^ f0); o1 = np.bitwise_or.reduce(a1 ^ f1)
    hb = first_bit(o0, o1); P = hb >> 3
    kb = np.zeros((len(a0), 16), np.int64)
    for j in range(16):
        kb[:, j] = ((a0 >> np.uint64(56 - 8 * j)) & np.uint64(255)).astype(np.int64) if j < 8 else ((a1 >> np.uint64(56 - 8 * (j - 8))) & np.uint64(255)).astype(np.int64)
    cs = []; nv = []
    for t in range(3):
        j = P + t
        col = kb[:, j] if j < 16 else np.zeros(len(a0), np.int64)
        pres = np.zeros(256, np.int64); pres[col] = 1
        rank = np.cumsum(pres) - pres
        cs.append(rank[col]); nv.append(pres.sum())
    N = nv[0] * nv[1] * nv[2]
    Mr = (512 << 32) // N if N > 512 else (1 << 32)
    x = (cs[0] * nv[1] + cs[1]) * nv[2] + cs[2]
    return (x * Mr) >> 32, nv
T = []; M = []; X = []; D = []; NV = []
for s in range(0, 200 * 20011, 20011):
    a0, a1 = k0[s:s + L], k1[s:s + L]
    dg, nv = scheme_code(a0, a1)
    t, m, x, d = trips(dg); T.append(t); M.append(m); X.append(x); D.append(d); NV.append(nv)
print(f"code  trips/leaf {np.mean(T):.1f}  mean bucket {np.mean(M):.2f}  max {np.mean(X):.1f} (worst {np.max(X)})  distinct {np.mean(D):.0f}")
print(NV[:10])
