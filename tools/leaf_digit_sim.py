import numpy as np, sys
rng = np.random.default_rng(1)
N = 4_000_000   # keys in one "partition" slice; leaves of ~256 consecutive sorted keys
alpha = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
K = alpha[rng.integers(0, 36, size=(N, 12))]
keys = np.sort(K.view('S12').ravel())
kb = np.frombuffer(keys.tobytes(), dtype=np.uint8).reshape(N, 12)
# big-endian 128-bit as two uint64 (k0 bytes 0..7, k1 bytes 8..11 then zero)
pad = np.zeros((N, 16), np.uint8); pad[:, :12] = kb
k0 = pad[:, :8].copy().view('>u8').ravel().astype(np.uint64)
k1 = pad[:, 8:].copy().view('>u8').ravel().astype(np.uint64)
def clz64(x):
    x = int(x)
    return 64 - x.bit_length()
def first_bit(o0, o1):
    return clz64(o0) if o0 else (64 + clz64(o1) if o1 else 128)
def bits_from(a0, a1, h, n):  # n bits starting at bit h from the top of the 128-bit key (vectorized)
    v = (a0.astype(object) << 64) | a1.astype(object)
    return np.array([(int(x) >> (128 - h - n)) & ((1 << n) - 1) if h + n <= 128 else (int(x) << (h + n - 128)) & ((1 << n) - 1) for x in v])
def key_bit(a0, a1, h):
    return ((a0 >> np.uint64(63 - h)) & np.uint64(1)).astype(np.int64) if h < 64 else ((a1 >> np.uint64(127 - h)) & np.uint64(1)).astype(np.int64)
def varying_digit(a0, a1, m0, m1, nb):
    # the first nb varying bits (mask m0:m1) of each key
    m = (int(m0) << 64) | int(m1)
    pos = [127 - i for i in range(128) if (m >> (127 - i)) & 1][:nb]  # bit index from LSB
    v = [(int(x) << 64) | int(y) for x, y in zip(a0, a1)]
    out = []
    for x in v:
        d = 0
        for p in pos: d = (d << 1) | ((x >> p) & 1)
        out.append(d << (nb - len(pos)))
    return np.array(out)
def scheme_old(a0, a1, varying=False):
    f0, f1 = a0[0], a1[0]
    o0 = np.bitwise_or.reduce(a0 ^ f0); o1 = np.bitwise_or.reduce(a1 ^ f1)
    hb = first_bit(o0, o1)
    sd = key_bit(a0, a1, hb); sf = sd[0]
    dg = np.zeros(len(a0), np.int64)
    for side in (0, 1):
        sel = sd == side
        if not sel.any(): continue
        r0, r1 = a0[sel][0], a1[sel][0]
        s0 = np.bitwise_or.reduce(a0[sel] ^ r0); s1 = np.bitwise_or.reduce(a1[sel] ^ r1)
        hs = min(first_bit(s0, s1), 120)
        if varying:
            dg[sel] = (side << 8) | varying_digit(a0[sel], a1[sel], s0, s1, 8)
        else:
            dg[sel] = (side << 8) | bits_from(a0[sel], a1[sel], hs, 8)
    return dg
def trips(dg):
    n = len(dg)
    cnt = np.bincount(dg, minlength=512)
    bn = cnt[dg]
    perm = rng.permutation(n)       # items sit in the leaf in random order
    bnp = bn[perm]
    t = 0
    for k in range(0, n, 64):
        t += bnp[k:k + 64].max()
    return t, bn.mean(), bn.max(), (cnt > 0).sum()
L = 256
for name, fn in [("old", lambda a, b: scheme_old(a, b)), ("side+varying8", lambda a, b: scheme_old(a, b, True))]:
    T = []; M = []; X = []; D = []
    for s in range(0, 200 * 20011, 20011):
        a0, a1 = k0[s:s + L], k1[s:s + L]
        t, m, x, d = trips(fn(a0, a1)); T.append(t); M.append(m); X.append(x); D.append(d)
    print(f"{name:16s} trips/leaf {np.mean(T):.1f}  mean bucket (per item) {np.mean(M):.2f}  max {np.mean(X):.1f}  distinct digits {np.mean(D):.0f}")
def scheme_var(a0, a1, nbits, skip=0):
    f0, f1 = a0[0], a1[0]
    o0 = np.bitwise_or.reduce(a0 ^ f0); o1 = np.bitwise_or.reduce(a1 ^ f1)
    hb = first_bit(o0, o1)
    sd = key_bit(a0, a1, hb)
    dg = np.zeros(len(a0), np.int64)
    for side in (0, 1):
        sel = sd == side
        if not sel.any(): continue
        r0, r1 = a0[sel][0], a1[sel][0]
        s0 = np.bitwise_or.reduce(a0[sel] ^ r0); s1 = np.bitwise_or.reduce(a1[sel] ^ r1)
        dg[sel] = (side << nbits) | varying_digit(a0[sel], a1[sel], s0, s1, nbits)
    return dg
def trips2(dg, nd):
    n = len(dg)
    cnt = np.bincount(dg, minlength=nd)
    bn = cnt[dg]
    perm = rng.permutation(n)
    bnp = bn[perm]
    return sum(bnp[k:k + 64].max() for k in range(0, n, 64)), bn.mean(), bn.max(), (cnt > 0).sum()
for nb in (8, 9, 10, 12, 16):
    T = []; M = []; X = []; D = []
    for s in range(0, 200 * 20011, 20011):
        a0, a1 = k0[s:s + L], k1[s:s + L]
        t, m, x, d = trips2(scheme_var(a0, a1, nb), 2 << nb); T.append(t); M.append(m); X.append(x); D.append(d)
    print(f"side+varying{nb:<3d} trips/leaf {np.mean(T):.1f}  mean bucket {np.mean(M):.2f}  max {np.mean(X):.1f}  distinct {np.mean(D):.0f}")
