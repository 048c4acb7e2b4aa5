// k_wide.hip -- high-cardinality ("wide") aggregation and formatting for gfx950 (BASELINE config C5).
//
// When most tokens miss the map kernel's LDS combine (near-unique keys), the reduce side of the
// reference -- sort every record by key (src/mr/worker.rs:162-164), group adjacent equal keys, call
// wc::reduce and write "{key} {count}\n" per group (worker.rs:165-184, src/app/wc.rs:15-17) -- is
// done by a two-level sample sort that moves each record three times instead of once per radix
// digit:
//   L1  records (16-byte packed keys) -> R x B1r buckets: partition r = SipHash-1-3(key) % R
//       (worker.rs:111-115, 129), then quantile splitters of a global sample (per-tile histogram,
//       scan, scatter);
//   L2  one workgroup per L1 bucket: quantile splitters of an 8 Ki sample of the bucket sorted in LDS,
//       histogram, scatter into leaves of ~1 Ki records;
//   leaf one workgroup per L1 bucket walks its leaves: an LDS hash table sums the leaf's records
//       (count 1) and the map tables' flushed counts (the "weighted" keys, pre-aggregated and sorted),
//       an LDS LSD radix sort over the key bytes that vary inside the leaf orders the distinct keys,
//       which are written in place with their counts, plus the leaf's line bytes;
//   write after a scan of the leaf byte totals (and the last-group drop of worker.rs:169-184 applied
//       to the last non-empty leaf of each partition), one workgroup per L1 bucket formats its
//       leaves' lines through LDS and stores them as whole dwords.
// Leaves whose distinct keys do not fit the LDS table (sample outliers, adversarial key sets) are
// listed and finished by a global radix sort of their records (mrgpu.cpp).
// Order within a leaf: (k0, k1) unsigned = key bytes (mrg_device.h), one partition per L1 bucket.
#include "mrg_device.h"
#include "mrg_internal.h"
#include "mrg_split.h"

namespace {

#define GASW __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ GASW T *gw(T *p) {
    return (GASW T *)p;
}

constexpr int W_WG = 1024;
constexpr int W_NW = W_WG / 64;
constexpr uint32_t W_S2 = 8192;       // L2 samples per L1 bucket (sorted in LDS)
#ifndef MRG_WIDE_L2U
#define MRG_WIDE_L2U 4   // L2 histogram: records per thread in flight
#endif
constexpr uint32_t W_L2D = 8192;          // SEG L2: digits
constexpr uint32_t W_L2DS = 2048;         // SEG L2: sampled records (the digit bytes' values)
constexpr uint32_t W_SCS = 6144;          // SEG L2: scatter chunk (above the stage: the leaf map, the leaves' ends)
constexpr uint32_t W_L2D_CNT = 32768;     // SEG L2: byte offset of the digit counts in the sample LDS
constexpr uint32_t W_L2D_MAP = 16u * W_SCS;   // SEG L2: byte offset of the digit -> leaf map
constexpr uint32_t W_L2D_END = W_L2D_MAP + 2u * W_L2D;   // SEG L2: byte offset of the leaves' region ends (u32)
constexpr uint32_t W_SC = 8192;       // L2 scatter chunk (staged in the samples' LDS)
constexpr int W_LWG = 256;            // leaf workgroup (four per CU: while one waits on memory, others work)
constexpr int W_LNW = W_LWG / 64;
constexpr uint32_t W_SLOTS = 1024;    // leaf LDS table slots
constexpr uint32_t W_MAXD = 768;      // distinct keys a leaf may hold (75 % load)
constexpr uint32_t W_SEGLDS = 2048;   // segment offsets cached in LDS per L1 tile
constexpr uint32_t W_MAXSEG = 512;    // segmented L2: map workgroups (segments per bucket) at most

// Workgroup barrier for LDS hand-offs only.  __syncthreads() also makes every wave wait for its
// outstanding global stores (vmcnt(0)) -- a store's full round trip at each of the many barriers of a
// leaf -- though no kernel here exchanges global data between its waves: only LDS needs ordering.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}


// ---------------------------------------------------------------- the map's records (count 1)
// main segments: the tail regions of 12-byte records (bucket-major, map workgroup minor), the
// per-bucket overflow lists, then the 16-byte tail regions (keys of 13..16 bytes) -- the order of
// mrg_launch_wmain_counts
__device__ __forceinline__ void main_rec(const BucketArgs &A, uint64_t s, uint64_t i, uint64_t &k0, uint64_t &k1) {
    const uint64_t nt = (uint64_t)A.nreg * MRG_NBUCKET;
    const GASW uint64_t *p;
    if (s < nt) {
        const uint32_t b = (uint32_t)(s / A.nreg), w = (uint32_t)(s % A.nreg);
        const GASW uint32_t *r = reinterpret_cast<const GASW uint32_t *>(
            reinterpret_cast<const GASW uint8_t *>(gw(A.pool)) + 12u * (A.rbase[b] + (uint64_t)w * A.bcap[b] + i));
        k0 = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
        k1 = (uint64_t)r[2] << 32;
        return;
    } else if (s < nt + MRG_NBUCKET) {
        p = gw(A.movf) + 2 * ((s - nt) * A.mocap + i);
    } else {
        const uint64_t s2 = s - nt - MRG_NBUCKET;
        const uint32_t b = (uint32_t)(s2 / A.nreg), w = (uint32_t)(s2 % A.nreg);
        p = gw(A.pool16) + 2 * (A.rbase16[b] + (uint64_t)w * A.bcap16[b] + i);
    }
    const uint64_t a = p[0], b = p[1];
    k0 = a;
    k1 = b;
}

// a record of a main segment whose first record is at `segptr` (bit 0 set: 12-byte records
// {k0, high word of k1}; clear: 16-byte records {k0, k1}); 12-byte segments have 4 bytes of slack
// after their last record, so both are one 16-byte load
typedef uint64_t v2w __attribute__((ext_vector_type(2)));
typedef uint32_t v4wu __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ void seg_rec(uint64_t segptr, uint64_t i, uint64_t &k0, uint64_t &k1) {
    const bool w12 = segptr & 1u;
    const uint64_t base = segptr & ~1ull;
    const v4wu x = *reinterpret_cast<const GASW v4wu *>((const GASW uint8_t *)(base + (w12 ? 12u : 16u) * i));
    k0 = (uint64_t)x.x | ((uint64_t)x.y << 32);
    k1 = w12 ? (uint64_t)x.z << 32 : ((uint64_t)x.z | ((uint64_t)x.w << 32));
}

// s in [lo, hi) with off[s] <= i < off[s + 1]  (off non-decreasing; empty segments are skipped)
template <class OFF>
__device__ __forceinline__ uint64_t seg_find(const OFF &off, uint64_t lo, uint64_t hi, uint64_t i) {
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (off(mid) <= i) lo = mid;
        else hi = mid;
    }
    return lo;
}


// number of splitters <= key among sp[0 .. m)
template <class SP>
__device__ __forceinline__ uint32_t upper_idx(const SP &sp, uint32_t m, uint64_t k0, uint64_t k1) {
    uint32_t lo = 0, hi = m;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        uint64_t s0, s1;
        sp(mid, s0, s1);
        if (key_lt(k0, k1, s0, s1)) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// segment sizes, and each segment's first record as an address (the L1 passes then read a record
// with one load instead of two dependent table lookups and a 64-bit division)
__global__ void k_wmain_counts(BucketArgs A, uint64_t *cnt, uint64_t *segptr) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nt = (uint64_t)A.nreg * MRG_NBUCKET;
    if (s < nt) {
        const uint32_t b = (uint32_t)(s / A.nreg), w = (uint32_t)(s % A.nreg);
        cnt[s] = min(A.bcount[(uint64_t)w * MRG_NBUCKET + b], A.bcap[b]);
        segptr[s] = (uint64_t)((const uint8_t *)A.pool + 12u * (A.rbase[b] + (uint64_t)w * A.bcap[b])) | 1u;
    } else if (s < nt + MRG_NBUCKET) {
        cnt[s] = min(A.monext[s - nt], A.mocap);
        segptr[s] = (uint64_t)(A.movf + 2 * ((s - nt) * A.mocap));
    } else if (s < 2 * nt + MRG_NBUCKET) {
        const uint64_t s2 = s - nt - MRG_NBUCKET;
        const uint32_t b = (uint32_t)(s2 / A.nreg), w = (uint32_t)(s2 % A.nreg);
        cnt[s] = min(A.bcount16[(uint64_t)w * MRG_NBUCKET + b], A.bcap16[b]);
        segptr[s] = (uint64_t)(A.pool16 + 2 * (A.rbase16[b] + (uint64_t)w * A.bcap16[b]));
    }
}

// flushed map tables: weighted entries (count fcnt) as plain arrays for the HBM-table aggregation
__global__ void k_wflush_counts(BucketArgs A, uint64_t *cnt) {
    const uint32_t w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w < A.nreg) cnt[w] = A.foff[(uint64_t)w * (MRG_NBUCKET + 1) + MRG_NBUCKET];
}
__global__ void k_wflush_gather(BucketArgs A, const uint64_t *off, uint64_t *k0, uint64_t *k1, uint32_t *c) {
    const uint32_t w = blockIdx.x;
    const uint64_t o = off[w], n = off[w + 1] - o;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint64_t j = (uint64_t)w * A.regcap + i;
        k0[o + i] = A.fk0[j];
        k1[o + i] = A.fk1[j];
        c[o + i] = A.fcnt[j];
    }
}

// ---------------------------------------------------------------- L1: sample, splitters
__global__ void k_wsample1(BucketArgs A, const uint64_t *off, uint64_t nseg, uint64_t n, uint32_t S, uint32_t R,
                           SortRec *out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= S) return;
    const uint64_t i = ((2ull * j + 1ull) * n) / (2ull * S);
    const uint64_t s = seg_find([&](uint64_t x) { return off[x]; }, 0, nseg, i);
    uint64_t k0, k1;
    main_rec(A, s, i - off[s], k0, k1);
    SortRec r;
    r.k0 = k0;
    r.k1 = k1;
    r.part = part_of(k0, k1, R);
    r.doc = 0;
    r.idx = j;
    r.pad = 0;
    out[j] = r;
}

// splitter q (< B1r - 1) of partition r: the sample at quantile (q + 1) / B1r of partition r's samples
__global__ void k_wsplit1(const SortRec *smp, uint32_t S, uint32_t R, uint32_t B1r, uint64_t *spl) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t m = B1r - 1u;
    if (t >= R * m) return;
    const uint32_t r = t / m, q = t % m;
    auto lower = [&](uint32_t p) {  // first sample with part >= p
        uint32_t lo = 0, hi = S;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (smp[mid].part < p) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    };
    const uint32_t lo = lower(r), hi = lower(r + 1u);
    uint64_t a = 0, b = 0;  // no sample: every key of r lands in the partition's last bucket
    if (hi > lo) {
        const uint32_t k = lo + (uint32_t)(((uint64_t)(q + 1u) * (hi - lo)) / B1r);
        const uint32_t kk = k < hi ? k : hi - 1u;
        a = smp[kk].k0;
        b = smp[kk].k1;
    }
    spl[2ull * t] = a;
    spl[2ull * t + 1] = b;
}

// ---------------------------------------------------------------- wide map: input sample, regions
// Sample j of S from the input text, for the wide map's L1 splitters and its near-unique test: the
// first token after byte (2j + 1) * total / 2S of the documents.  The key is approximated on ASCII
// classes (bytes >= 0x80 count as word bytes, ASCII punctuation is dropped, the first 16 key bytes):
// splitters only steer bucket sizes, so any key-ordered value is a valid one (exactness comes from
// the map itself).
__global__ void k_wsample_text(const uint8_t *in, const uint64_t *doc_off, uint32_t n_docs, uint64_t total,
                               uint32_t S, uint32_t R, SortRec *out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= S) return;
    const uint64_t g = ((2ull * j + 1ull) * total) / (2ull * S);
    uint32_t lo = 0, hi = n_docs;  // doc_off[lo] - doc_off[0] <= g < ...
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (doc_off[mid] - doc_off[0] <= g) lo = mid;
        else hi = mid;
    }
    const uint64_t dhi = doc_off[lo + 1];
    uint64_t p = doc_off[0] + g;
    auto cls = [](uint32_t c) -> uint32_t {  // 0 space, 1 word byte, 2 other (deleted)
        if (c >= 0x80u) return 1u;
        const uint32_t k = mrg_uclass(c);
        return k == MRG_CLS_S ? 0u : (k == MRG_CLS_W ? 1u : 2u);
    };
    for (int k = 0; k < 64 && p < dhi && cls(in[p]) != 0u; ++k) ++p;  // the rest of the current token
    for (int k = 0; k < 64 && p < dhi && cls(in[p]) == 0u; ++k) ++p;  // the separator
    uint64_t k0 = 0, k1 = 0;
    uint32_t L = 0;
    for (int k = 0; k < 64 && p < dhi && L < 16u; ++k, ++p) {
        const uint32_t c = in[p], t = cls(c);
        if (t == 0u) break;
        if (t == 1u) mrg_key_append(k0, k1, L++, c);
    }
    SortRec r;
    r.k0 = k0;
    r.k1 = k1;
    r.part = L ? part_of(k0, k1, R) : 0u;
    r.doc = 0;
    r.idx = j;
    r.pad = 0;
    out[j] = r;
}

// sorted samples: adjacent equal keys (the near-unique test) in dups[0], keys of 13..16 bytes in dups[1]
__global__ void k_wsample_dups(const SortRec *r, uint32_t S, unsigned long long *dups) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    const bool d = j > 0 && j < S && r[j].part == r[j - 1].part && r[j].k0 == r[j - 1].k0 && r[j].k1 == r[j - 1].k1;
    const bool w16 = j < S && (uint32_t)r[j].k1 != 0u;
    const uint64_t m = __ballot(d), m16 = __ballot(w16);
    if ((threadIdx.x & 63u) == 0 && m) atomicAdd(dups, (unsigned long long)__popcll(m));
    if ((threadIdx.x & 63u) == 0 && m16) atomicAdd(dups + 1, (unsigned long long)__popcll(m16));
}

// The cold-context decision (r06): S <= W_UQ / 2 unsorted samples, one workgroup, an LDS set of 64-bit
// fingerprints of (part, key): dups[0] = samples whose fingerprint an earlier sample already holds (= S -
// distinct, the sorted test's adjacent-equal count up to fingerprint collisions: a heuristic either way),
// dups[1] = keys of 13..16 bytes.  One launch and no sort, so a job on text with repeats pays ~20 us for
// the test instead of the full sample's radix sort.
constexpr uint32_t W_UQ = 16384;
__global__ __launch_bounds__(1024) void k_wsample_uniq(const SortRec *r, uint32_t S, unsigned long long *dups) {
    __shared__ unsigned long long s_fp[W_UQ];
    __shared__ unsigned int s_n[2];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < W_UQ; i += 1024u) s_fp[i] = 0ull;
    if (tid < 2u) s_n[tid] = 0u;
    __syncthreads();
    uint32_t nd = 0, n16 = 0;
    for (uint32_t j = tid; j < S; j += 1024u) {
        const SortRec x = r[j];
        const uint64_t fp = mrg_fmix64(x.k0 ^ mrg_fmix64(x.k1 ^ ((uint64_t)x.part << 32))) | 1ull;   // never 0 (= empty)
        n16 += (uint32_t)x.k1 != 0u ? 1u : 0u;
        uint32_t h = (uint32_t)(fp >> 40) & (W_UQ - 1u);
        for (uint32_t k = 0; k < W_UQ; ++k, h = (h + 1u) & (W_UQ - 1u)) {
            const unsigned long long old = atomicCAS(&s_fp[h], 0ull, (unsigned long long)fp);
            if (old == 0ull) break;
            if (old == fp) { ++nd; break; }
        }
    }
    if (nd) atomicAdd(&s_n[0], nd);
    if (n16) atomicAdd(&s_n[1], n16);
    __syncthreads();
    if (tid == 0) {
        dups[0] = s_n[0];
        dups[1] = s_n[1];
    }
}

struct L1Args {
    BucketArgs A;
    const uint64_t *off;     // main segment offsets [nseg + 1]
    const uint64_t *segptr;  // [nseg] address of each segment's first record
    uint64_t nseg, n;
    const uint64_t *spl1;    // [R][B1r - 1] (k0, k1)
    uint32_t R, B1r, B1, ntiles;
    uint32_t *cnt;           // [B1][ntiles] (scanned in place between the two kernels)
    uint64_t *out;           // L1 output, 2 words per record
    uint16_t *bid;           // [n] L1 bucket of each record: written by the counting pass, read by the scatter
    const uint8_t *ix1;      // counting pass: per-partition splitter index [R][W_IX1] (null: binary search)
};

// L1 splitter index of partition r: 257 entries, then the prefix bit count (L1Index)
constexpr uint32_t W_IX1 = MRG_WIDE_IX1;
__global__ void k_wl1ix(const uint64_t *spl1, uint32_t m, uint8_t *ix1) {
    const uint32_t r = blockIdx.x;
    const uint64_t *sp = spl1 + 2ull * r * m;
    L1Index::build(sp, m, ix1 + (uint64_t)r * W_IX1, threadIdx.x, blockDim.x);
    if (threadIdx.x == 0) ix1[(uint64_t)r * W_IX1 + 257] = (uint8_t)L1Index::prefix_bits(sp, m);
}

// L1 tile t: records [t * T1, min(n, (t+1) * T1)); WITH_SCATTER: write them, else count them
template <bool SCATTER>
__global__ __launch_bounds__(W_WG, 1) void k_wl1(L1Args L) {
    extern __shared__ uint64_t s_dyn[];  // spl1 (2 * R * (B1r-1) u64) | hist (B1 u32) | seg offsets | seg ptrs
    uint64_t *s_spl = s_dyn;
    const uint32_t m = L.B1r - 1u;
    uint32_t *s_h = reinterpret_cast<uint32_t *>(s_spl + 2ull * L.R * m);
    uint64_t *s_off = reinterpret_cast<uint64_t *>(s_h + ((L.B1 + 1u) & ~1u));
    uint64_t *s_ptr = s_off + W_SEGLDS;
    uint8_t *s_ix = reinterpret_cast<uint8_t *>(s_ptr + W_SEGLDS);   // [R][W_IX1] if L.ix1
    __shared__ uint64_t s_lo, s_hi;
    const uint32_t tid = threadIdx.x, t = blockIdx.x;
    const uint64_t t0 = (uint64_t)t * MRG_WIDE_T1, t1 = min(L.n, t0 + MRG_WIDE_T1);
    for (uint32_t i = tid; i < 2u * L.R * m; i += W_WG) s_spl[i] = L.spl1[i];
    for (uint32_t b = tid; b < L.B1; b += W_WG) s_h[b] = SCATTER ? L.cnt[(uint64_t)b * L.ntiles + t] : 0u;
    if (!SCATTER && L.ix1)
        for (uint32_t i = tid; i < L.R * (W_IX1 / 4); i += W_WG)
            reinterpret_cast<uint32_t *>(s_ix)[i] = reinterpret_cast<const uint32_t *>(L.ix1)[i];
    if (tid == 0) {
        const auto off = [&](uint64_t x) { return L.off[x]; };
        s_lo = seg_find(off, 0, L.nseg, t0);
        s_hi = seg_find(off, 0, L.nseg, t1 - 1u) + 1u;
    }
    lds_barrier();
    const uint64_t slo = s_lo, shi = s_hi;
    const bool cached = shi - slo + 1u <= W_SEGLDS;
    if (cached)
        for (uint64_t x = slo + tid; x <= shi; x += W_WG) {
            s_off[x - slo] = L.off[x];
            if (x < shi) s_ptr[x - slo] = L.segptr[x];
        }
    lds_barrier();
    // U records per thread per round: their loads are all in flight before the first is used.
    // A thread visits its records in increasing order, so it keeps its segment (first record, end,
    // base address) in registers and only steps to the next segment when a record crosses its end:
    // no per-record search (three dependent LDS reads before every load).
    constexpr int U = 4;
    auto seg_off = [&](uint64_t x) -> uint64_t { return cached ? s_off[x - slo] : L.off[x]; };
    auto seg_ptr = [&](uint64_t x) -> uint64_t { return cached ? s_ptr[x - slo] : L.segptr[x]; };
    uint64_t sg = seg_find(seg_off, slo, shi, min(t0 + tid, t1 - 1u));
    uint64_t seg_lo = seg_off(sg), seg_hi = seg_off(sg + 1);
    uint64_t seg_p = seg_ptr(sg);
    for (uint64_t base = t0 + tid; base < t1; base += (uint64_t)U * W_WG) {
        uint64_t k0[U], k1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = min(base + (uint64_t)u * W_WG, t1 - 1u);  // past the tile: a repeat, unused
            while (i >= seg_hi) {  // rare: the next non-empty segment
                ++sg;
                seg_lo = seg_hi;
                seg_hi = seg_off(sg + 1);
                seg_p = seg_ptr(sg);
            }
            seg_rec(seg_p, i - seg_lo, k0[u], k1[u]);
        }
        uint32_t bk[U];
        if (SCATTER) {   // the bucket the counting pass found (no SipHash, no splitter search again)
#pragma unroll
            for (int u = 0; u < U; ++u) bk[u] = gw(L.bid)[min(base + (uint64_t)u * W_WG, t1 - 1u)];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (base + (uint64_t)u * W_WG >= t1) break;
            uint32_t b;
            if (SCATTER) {
                b = bk[u];
            } else {
                const uint32_t r = part_of(k0[u], k1[u], L.R);
                uint32_t q;
                if (L.ix1) {
                    const uint8_t *ixr = s_ix + r * W_IX1;
                    const L1Index li{s_spl + 2ull * r * m, ixr, m, ixr[257]};
                    q = li.upper(k0[u], k1[u]);
                } else {
                    q = upper_idx(
                        [&](uint32_t x, uint64_t &a, uint64_t &c) {
                            a = s_spl[2ull * (r * m + x)];
                            c = s_spl[2ull * (r * m + x) + 1];
                        },
                        m, k0[u], k1[u]);
                }
                b = r * L.B1r + q;
                gw(L.bid)[base + (uint64_t)u * W_WG] = (uint16_t)b;
            }
            const uint32_t pos = atomicAdd(&s_h[b], 1u);
            if (SCATTER) {
                typedef uint64_t v2 __attribute__((ext_vector_type(2)));
                *reinterpret_cast<GASW v2 *>(gw(L.out) + 2ull * pos) = v2{k0[u], k1[u]};
            }
        }
    }
    if (!SCATTER) {
        lds_barrier();
        for (uint32_t b = tid; b < L.B1; b += W_WG) L.cnt[(uint64_t)b * L.ntiles + t] = s_h[b];
    }
}

// bucket b starts at the scanned count of (b, tile 0); bstart[B1] = n
__global__ void k_wbstart(const uint32_t *cnt, uint32_t B1, uint32_t ntiles, uint64_t n, uint64_t *bstart) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < B1) bstart[b] = cnt[(uint64_t)b * ntiles];
    else if (b == B1) bstart[b] = n;
}

// ---------------------------------------------------------------- block helpers (1024 threads)
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t v) {
    const uint32_t lane = __lane_id();
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(v, o);
        if (lane >= o) v += u;
    }
    return v;
}
// exclusive block scan of one value per thread; s_ws holds NW words; *total = sum
template <int NW = W_NW>
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t *s_ws, uint32_t *total) {
    const uint32_t lane = __lane_id(), w = threadIdx.x >> 6;
    const uint32_t inc = wave_scan_incl(v);
    if (lane == 63) s_ws[w] = inc;
    lds_barrier();
    uint32_t base = 0, tot = 0;
    for (uint32_t i = 0; i < (uint32_t)NW; ++i) {
        const uint32_t x = s_ws[i];
        base += i < w ? x : 0u;
        tot += x;
    }
    lds_barrier();
    *total = tot;
    return base + inc - v;
}

// wide map regions of bucket b (one wave): segment starts soff[b][w] (bucket-relative; a region holds
// its count clipped to the capacity), w = grid the bucket's 16-byte list (12-byte regions only), then
// the bucket's total, also in nb[b]
__global__ __launch_bounds__(64) void k_wmap_seg(const uint32_t *wcnt, uint32_t grid, uint32_t wcap,
                                                 const uint32_t *wl16n, uint32_t wl16cap, uint32_t *soff, uint64_t *nb) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const uint32_t *c = wcnt + (uint64_t)b * grid;
    uint32_t *so = soff + (uint64_t)b * (grid + 2u);
    uint32_t run = 0;
    for (uint32_t w0 = 0; w0 < grid; w0 += 64) {
        const uint32_t w = w0 + lane;
        const uint32_t v = w < grid ? min(c[w], wcap) : 0u;
        const uint32_t inc = wave_scan_incl(v);
        if (w < grid) so[w] = run + inc - v;
        run += (uint32_t)__shfl(inc, 63);
    }
    if (lane == 0) {
        so[grid] = run;
        run += wl16n ? min(wl16n[b], wl16cap) : 0u;
        so[grid + 1] = run;
        nb[b] = run;
    }
}

// ---------------------------------------------------------------- L2: per L1 bucket
struct L2Args {
    const uint64_t *in;      // L1 output (2 words per record)
    uint64_t *out;           // leaf order (2 words per record)
    const uint64_t *bstart;  // [B1 + 1]
    const uint64_t *spl1;
    uint32_t B1r, target;
    uint32_t *nleaf;         // [B1]
    uint64_t *leaf_lo;       // [B1 * MAXB2 + 1] first record of each leaf in `out` (absolute)
    uint64_t *leaf_hi;       // [B1 * MAXB2] one past its last record in `out`
    uint64_t *leaf_dlo;      // [B1 * MAXB2] its first record in the dense order (bstart-based): output slots
    uint64_t *leaf_lb;       // [B1 * MAXB2][2] lower key bound of each leaf
    uint16_t *sub;           // [n] leaf (inside its L1 bucket) of each record: histogram pass -> scatter
    // segmented input (the wide map's regions): L1 bucket b's records are segments w <= grid at
    // bucket-relative offsets soff[b * (grid + 2) + w]: w < grid the region of (b, w), records
    // [(b * grid + w) * wcap, + its count) of rin (12 bytes each when w12, else 16), w = grid the
    // bucket's list of 16-byte records (wl16 [b * wl16cap, ...); empty unless w12)
    const uint64_t *rin;
    const uint32_t *soff;
    uint32_t grid, wcap, w12, wl16cap;
    const uint64_t *wl16;
    // sparse leaves (SEG only, r06): bucket b's leaves live in out [9 bstart[b] / 4, 9 bstart[b + 1] / 4);
    // the histogram counts a quarter of each segment, leaf j gets capmul * (its sampled records) +
    // capadd slots, and a bucket whose leaf overflows is redone with the exact histogram
    uint32_t sparse, capmul, capadd;
    uint32_t sample_min;      // buckets of fewer records take the exact histogram at once
    uint32_t redo;            // the redo launch: only buckets with redo_flags[b] set, exact histogram
    uint32_t *redo_flags;     // [B1] buckets whose sampled leaves overflowed (zeroed by the host)
};

// record r of segment w of bucket b (segmented input), as (k0, k1)
typedef uint32_t v4wua __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ void seg_load(const L2Args &L, uint32_t b, uint32_t w, uint64_t r, uint64_t &k0,
                                         uint64_t &k1) {
    if (w == L.grid) {
        const GASW uint64_t *p = gw(L.wl16) + 2ull * ((uint64_t)b * L.wl16cap + r);
        k0 = p[0];
        k1 = p[1];
        return;
    }
    const uint64_t i = ((uint64_t)b * L.grid + w) * L.wcap + r;
    if (L.w12) {  // one 16-byte load (4 bytes of slack after the last region)
        const v4wua x = *reinterpret_cast<const GASW v4wua *>(reinterpret_cast<const GASW uint8_t *>(gw(L.rin)) + 12u * i);
        k0 = (uint64_t)x.x | ((uint64_t)x.y << 32);
        k1 = (uint64_t)x.z << 32;
    } else {
        const GASW uint64_t *p = gw(L.rin) + 2ull * i;
        k0 = p[0];
        k1 = p[1];
    }
}

// Segmented input: record i (bucket-relative) of bucket b, through its segment (binary search)
__device__ __forceinline__ void seg_record(const L2Args &L, uint32_t b, const uint32_t *so, uint64_t i, uint64_t &k0,
                                           uint64_t &k1) {
    uint32_t lo = 0, hi = L.grid + 1u;  // so[lo] <= i < so[hi]
    while (hi - lo > 1u) {
        const uint32_t mid = (lo + hi) >> 1;
        if (so[mid] <= i) lo = mid;
        else hi = mid;
    }
    seg_load(L, b, lo, i - so[lo], k0, k1);
}

// byte j (0 = most significant) of a packed key, 0 past byte 15
__device__ __forceinline__ uint32_t key_byte(uint64_t k0, uint64_t k1, uint32_t j) {
    return j < 8u ? (uint32_t)(k0 >> (56u - 8u * j)) & 0xFFu : (j < 16u ? (uint32_t)(k1 >> (56u - 8u * (j - 8u))) & 0xFFu : 0u);
}
#ifdef MRG_WIDE_PROF  // diagnostic build: L2 phase clocks of thread 0 of every workgroup
__device__ unsigned long long g_l2prof[8];
#define L2P(i) { if (tid == 0) { const uint64_t t_ = clock64(); l2acc[i] += t_ - l2t; l2t = t_; } }
#else
#define L2P(i)
#endif
template <bool SEG>
__global__ __launch_bounds__(W_WG, 1) void k_wl2(L2Args L) {
    __shared__ uint64_t s_smp[2 * W_S2];            // samples (k0, k1), bitonic-sorted
    __shared__ uint64_t s_spl[2 * MRG_WIDE_MAXB2];  // (one spare pair: the scatter's leaf ids fill it all)
    __shared__ uint32_t s_cnt[MRG_WIDE_MAXB2];
    __shared__ uint32_t s_cur[MRG_WIDE_MAXB2];
    __shared__ uint32_t s_bst[MRG_WIDE_MAXB2];      // scatter: a chunk's leaf starts
    static_assert(W_SC * sizeof(uint64_t) * 2 <= sizeof(s_smp) && W_SC * sizeof(uint16_t) <= sizeof(s_spl),
                  "the scatter's stage fits the sample and splitter arrays");
    static_assert(16 * W_L2DS <= W_L2D_CNT && W_L2D_CNT + 4 * W_L2D <= W_L2D_MAP && W_L2D_END + 4 * MRG_WIDE_MAXB2 <= sizeof(s_smp) &&
                  W_SCS * sizeof(uint16_t) <= sizeof(s_spl) && W_L2D % W_WG == 0,
                  "SEG L2: samples, digit counts, leaf map and stage fit the sample LDS");
    __shared__ uint32_t s_ws[W_NW];
    __shared__ uint32_t s_cseg[SEG ? W_MAXSEG + 2 : 1];   // SEG: the bucket's segment starts
    __shared__ uint32_t s_dor[SEG ? 4 : 1];                // SEG: OR of the samples' bits against the first
    __shared__ uint32_t s_dnv[SEG ? 4 : 1];                // SEG: values present at the three digit bytes
    __shared__ uint16_t s_dcode[SEG ? 3 * 256 : 1];        // SEG: the digit bytes' codes (live through the scatter)
    const uint32_t tid = threadIdx.x, b = blockIdx.x;
    if (SEG && L.redo && L.redo_flags[b] == 0u) return;   // (uniform) only flagged buckets are redone
#ifdef MRG_WIDE_PROF
    uint64_t l2acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, l2t = clock64();
#endif
    if (SEG) {
        for (uint32_t w = tid; w <= L.grid + 1u; w += W_WG) s_cseg[w] = L.soff[(uint64_t)b * (L.grid + 2u) + w];
        lds_barrier();
    }
    L2P(0);
    const uint64_t base = L.bstart[b], nb = L.bstart[b + 1] - base;
    uint32_t B2 = (uint32_t)min<uint64_t>((nb + L.target - 1) / L.target, MRG_WIDE_MAXB2);
    if (B2 < 1) B2 = 1;
    const GASW uint64_t *in = gw(L.in) + 2 * base;
    // SEG (the wide map's buckets): leaves are runs of DIGITS, not ranges between sampled splitters.
    // digit = the key bytes P, P + 1, P + 2 from the first byte the bucket's keys may differ on (the
    // sample's, bounded by the bucket's splitters), each replaced by its rank among the values a
    // sample shows at that byte, in mixed radix scaled to W_L2D digits (a value the sample lacks:
    // see the radices below; profiles/r05 and tools/leaf_digit_sim*.py check the order).
    // The histogram counts digits; a leaf = the digits whose running count falls in one multiple of
    // the target.  No sample sort, and leaves come out the target size (a digit holds ~31 records
    // at C5) instead of varying like 8-sample gaps (4 % of them went to the workgroup kernel).
    uint32_t *dcnt = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(s_smp) + W_L2D_CNT);
    uint16_t *lmap = reinterpret_cast<uint16_t *>(reinterpret_cast<uint8_t *>(s_smp) + W_L2D_MAP);
    uint16_t *dcode = s_dcode;   // [3][256]: 2 x (values present below) + present
    uint32_t dP = 0, dn1 = 1, dn2 = 1;
    uint64_t dM = 1ull << 32;
    uint64_t dtgt = L.target;
    if (SEG) {
        dtgt = max<uint64_t>(L.target, (nb + MRG_WIDE_MAXB2 - 1) / MRG_WIDE_MAXB2);
        B2 = nb ? (uint32_t)((nb - 1) / dtgt + 1) : 1u;
    }
    // ---- splitters from a sorted sample
    if (SEG && B2 > 1) {
        const uint32_t S = (uint32_t)min<uint64_t>(nb, W_L2DS);
        if (tid < 4) s_dor[tid] = 0;
        for (uint32_t i = tid; i < 3u * 128u; i += W_WG) reinterpret_cast<uint32_t *>(dcode)[i] = 0;
        for (uint32_t i = tid; i < W_L2D; i += W_WG) dcnt[i] = 0;
        for (uint32_t k = tid; k < S; k += W_WG) {
            uint64_t a, c;
            seg_record(L, b, s_cseg, ((2ull * k + 1ull) * nb) / (2ull * S), a, c);
            s_smp[2 * k] = a;
            s_smp[2 * k + 1] = c;
        }
        lds_barrier();
        {
            const uint64_t f0 = s_smp[0], f1 = s_smp[1];
            uint64_t o0 = 0, o1 = 0;
            for (uint32_t k = tid; k < S; k += W_WG) {
                o0 |= s_smp[2 * k] ^ f0;
                o1 |= s_smp[2 * k + 1] ^ f1;
            }
            for (int o = 32; o > 0; o >>= 1) {
                o0 |= __shfl_xor(o0, o);
                o1 |= __shfl_xor(o1, o);
            }
            if ((tid & 63u) == 0) {
                if (o0) { atomicOr(&s_dor[0], (uint32_t)o0); atomicOr(&s_dor[1], (uint32_t)(o0 >> 32)); }
                if (o1) { atomicOr(&s_dor[2], (uint32_t)o1); atomicOr(&s_dor[3], (uint32_t)(o1 >> 32)); }
            }
        }
        lds_barrier();
        {
            // P: the first byte the sample differs on, but no later than the first byte the bucket's
            // bounds differ on -- keys outside the sample may differ earlier than it, never earlier
            // than the bounds (every key lies between them)
            uint64_t o0 = (uint64_t)s_dor[0] | ((uint64_t)s_dor[1] << 32), o1 = (uint64_t)s_dor[2] | ((uint64_t)s_dor[3] << 32);
            const uint32_t q = b % L.B1r, r = b / L.B1r;
            const uint64_t *sp = L.spl1 + 2ull * r * (L.B1r - 1u);
            const uint64_t l0 = q > 0 ? sp[2 * (q - 1u)] : 0ull, l1 = q > 0 ? sp[2 * (q - 1u) + 1] : 0ull;
            const uint64_t h0 = q + 1u < L.B1r ? sp[2 * q] : ~0ull, h1 = q + 1u < L.B1r ? sp[2 * q + 1] : ~0ull;
            o0 |= l0 ^ h0;
            o1 |= l1 ^ h1;
            const uint32_t hb = o0 ? (uint32_t)__builtin_clzll(o0) : (o1 ? 64u + (uint32_t)__builtin_clzll(o1) : 0u);
            dP = hb >> 3;
        }
        for (uint32_t k = tid; k < S; k += W_WG) {
            const uint64_t a = s_smp[2 * k], c = s_smp[2 * k + 1];
#pragma unroll
            for (uint32_t t = 0; t < 3; ++t) dcode[256u * t + key_byte(a, c, dP + t)] = 1;
        }
        lds_barrier();
        if (tid < 3u * 64u) {   // presence -> 2 x (present values below v) + (v present)
            const uint32_t t = tid >> 6, lane = tid & 63u;
            uint32_t *cw = reinterpret_cast<uint32_t *>(dcode + 256u * t);
            const uint32_t w0 = cw[2 * lane], w1 = cw[2 * lane + 1];   // values 4 lane .. 4 lane + 3
            const uint32_t pr[4] = {w0 & 1u, w0 >> 16, w1 & 1u, w1 >> 16};
            const uint32_t cnt = pr[0] + pr[1] + pr[2] + pr[3];
            const uint32_t inc = wave_scan_incl(cnt);
            uint32_t run = inc - cnt, e[4];
#pragma unroll
            for (uint32_t x = 0; x < 4; ++x) {
                e[x] = (run << 1) | pr[x];
                run += pr[x];
            }
            cw[2 * lane] = e[0] | (e[1] << 16);
            cw[2 * lane + 1] = e[2] | (e[3] << 16);
            if (lane == 63) s_dnv[t] = inc;
        }
        lds_barrier();
        // radices n + 1: a value the sample lacks takes the code of the next present value (or n)
        // and zeroes the less significant codes, so the digit never decreases along the key order
        // (a lacking value collapsed onto a present one, with its lower bytes kept, would reorder)
        const uint64_t N = (uint64_t)(s_dnv[0] + 1u) * (s_dnv[1] + 1u) * (s_dnv[2] + 1u);
        dn1 = s_dnv[1] + 1u;
        dn2 = s_dnv[2] + 1u;
        dM = N > W_L2D ? ((uint64_t)W_L2D << 32) / N : (1ull << 32);
    } else if (!SEG && B2 > 1) {
        const uint32_t S = (uint32_t)min<uint64_t>(nb, W_S2);
        uint32_t P = 1;
        while (P < S) P <<= 1;
        for (uint32_t k = tid; k < P; k += W_WG) {
            uint64_t a = ~0ull, c = ~0ull;  // padding sorts last
            if (k < S) {
                const uint64_t i = ((2ull * k + 1ull) * nb) / (2ull * S);
                if (SEG) {
                    seg_record(L, b, s_cseg, i, a, c);
                } else {
                    a = in[2 * i];
                    c = in[2 * i + 1];
                }
            }
            s_smp[2 * k] = a;
            s_smp[2 * k + 1] = c;
        }
        lds_barrier();
        L2P(1);
        for (uint32_t size = 2; size <= P; size <<= 1) {
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t t = tid; t < P / 2; t += W_WG) {
                    const uint32_t i = 2 * t - (t & (stride - 1));  // low element of the pair
                    const uint32_t j = i + stride;
                    const bool up = (i & size) == 0;
                    const uint64_t a0 = s_smp[2 * i], a1 = s_smp[2 * i + 1], b0 = s_smp[2 * j], b1 = s_smp[2 * j + 1];
                    if (key_lt(b0, b1, a0, a1) == up) {
                        s_smp[2 * i] = b0; s_smp[2 * i + 1] = b1;
                        s_smp[2 * j] = a0; s_smp[2 * j + 1] = a1;
                    }
                }
                lds_barrier();
            }
        }
        L2P(2);
        for (uint32_t q = tid; q + 1 < B2; q += W_WG) {
            const uint32_t k = (uint32_t)(((uint64_t)(q + 1u) * S) / B2);
            s_spl[2 * q] = s_smp[2 * k];
            s_spl[2 * q + 1] = s_smp[2 * k + 1];
        }
        lds_barrier();
        // the sample is dead now: its LDS holds the splitter index
        LeafIndex::build(s_spl, B2 - 1u, reinterpret_cast<uint16_t *>(s_smp), tid, W_WG);
    }
    const LeafIndex si{s_spl, reinterpret_cast<const uint16_t *>(s_smp), B2 - 1u,
                       (!SEG && B2 > 1) ? LeafIndex::prefix_bits(s_spl, B2 - 1u) : 0u};
    auto sub_of = [&](uint64_t k0, uint64_t k1) -> uint32_t {
        if (SEG) {
            if (B2 <= 1) return 0u;
            const uint32_t e0 = dcode[key_byte(k0, k1, dP)], e1 = dcode[256u + key_byte(k0, k1, dP + 1u)],
                           e2 = dcode[512u + key_byte(k0, k1, dP + 2u)];
            const uint32_t c1 = (e0 & 1u) ? e1 >> 1 : 0u, c2 = (e0 & e1 & 1u) ? e2 >> 1 : 0u;
            const uint32_t x = ((e0 >> 1) * dn1 + c1) * dn2 + c2;
            return (uint32_t)(((uint64_t)x * dM) >> 32);
        }
        return B2 > 1 ? si.upper(k0, k1) : 0u;
    };
    L2P(3);
    // sparse leaves (SEG, large buckets): the histogram counts a quarter of every segment and each leaf
    // gets a region of capmul x its sampled records + capadd; a bucket whose leaf overflows its region
    // (or whose capacities pass the bucket's budget) is flagged and redone with the exact histogram by
    // a second launch (L.redo: the other buckets' workgroups return at once)
    uint32_t *s_end = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(s_smp) + W_L2D_END);
    __shared__ uint32_t s_ovf;
    const bool sparse = SEG && L.sparse != 0u;
    const uint64_t obase = sparse ? 9u * base / 4u : base;
    const uint64_t obud = sparse ? 9u * (base + nb) / 4u - obase : nb;   // slots of this bucket in `out`
    const bool samp = sparse && !L.redo && B2 > 1 && nb >= L.sample_min;
    const uint64_t dtg = samp ? max<uint64_t>(1u, dtgt / 4u) : dtgt;
    for (uint32_t j = tid; j < MRG_WIDE_MAXB2; j += W_WG) {
        s_cnt[j] = 0;
        s_cur[j] = 0;
    }
    if (tid == 0) s_ovf = 0u;
    lds_barrier();
    // ---- histogram (U records per thread in flight)
    constexpr int U = MRG_WIDE_L2U;
    typedef uint64_t v2 __attribute__((ext_vector_type(2)));
    const GASW v2 *inv = reinterpret_cast<const GASW v2 *>(in);
    if (SEG) {  // segment by segment, one wave each: reads stay inside a segment
        const uint32_t *so = s_cseg;
        const uint32_t lane = tid & 63u;
        for (uint32_t w = tid >> 6; w <= L.grid; w += W_NW) {
            const uint32_t o = so[w], nwa = so[w + 1] - o;
            const uint32_t nw = samp ? (nwa + 3u) / 4u : nwa;   // sampled: the segment's first quarter
            for (uint32_t j0 = lane; j0 < nw; j0 += (uint32_t)U * 64u) {
                v2 x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    uint64_t a, c;
                    seg_load(L, b, w, min(j0 + (uint32_t)u * 64u, nw - 1u), a, c);
                    x[u] = v2{a, c};
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (j0 + (uint32_t)u * 64u < nw) {
                        const uint32_t j = sub_of(x[u].x, x[u].y);
                        atomicAdd(B2 > 1 ? &dcnt[j] : &s_cnt[0], 1u);   // SEG: digits
                        if (!SEG) gw(L.sub)[base + o + j0 + (uint64_t)u * 64u] = (uint16_t)j;   // SEG: recomputed
                    }
            }
        }
    } else {
        for (uint64_t i0 = tid; i0 < nb; i0 += (uint64_t)U * W_WG) {
            v2 x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = inv[min(i0 + (uint64_t)u * W_WG, (uint64_t)(nb - 1u))];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (i0 + (uint64_t)u * W_WG < nb) {
                    const uint32_t j = sub_of(x[u].x, x[u].y);
                    atomicAdd(&s_cnt[j], 1u);
                    gw(L.sub)[base + i0 + (uint64_t)u * W_WG] = (uint16_t)j;
                }
        }
    }
    lds_barrier();
    if (SEG && B2 > 1) {   // digit d -> leaf floor(records before d / target); the leaves' counts
        constexpr uint32_t PT = W_L2D / W_WG;
        uint32_t v[PT], sum = 0;
#pragma unroll
        for (uint32_t x = 0; x < PT; ++x) {
            v[x] = dcnt[tid * PT + x];
            sum += v[x];
        }
        uint32_t tot;
        uint32_t run = block_scan_excl(sum, s_ws, &tot);
#pragma unroll
        for (uint32_t x = 0; x < PT; ++x) {
            const uint32_t leaf = min((uint32_t)(run / dtg), B2 - 1u);
            lmap[tid * PT + x] = (uint16_t)leaf;
            if (v[x]) atomicAdd(&s_cnt[leaf], v[x]);
            run += v[x];
        }
        lds_barrier();
    }
    L2P(4);
    {  // exclusive scan of the B2 <= 1024 counts (sampled: region capacities), one per thread
        const uint32_t v = tid < B2 ? (samp ? L.capmul * s_cnt[tid] + L.capadd : s_cnt[tid]) : 0u;
        uint32_t tot;
        const uint32_t ex = block_scan_excl(v, s_ws, &tot);
        if (tid < B2) {
            s_cur[tid] = ex;
            if (SEG) s_end[tid] = ex + v;
        }
        if (tid == 0) s_ovf = samp && (uint64_t)tot > obud ? 1u : 0u;   // capacities past the budget: exact
        const uint64_t lid = (uint64_t)b * MRG_WIDE_MAXB2 + tid;
        if (tid < B2) {
            L.leaf_lo[lid] = obase + ex;
            uint64_t a, c;
            if (SEG) {   // digit leaves have no key bound (the wide map's job has no weighted keys)
                a = 0;
                c = 0;
            } else if (tid > 0) {
                a = s_spl[2 * (tid - 1)];
                c = s_spl[2 * (tid - 1) + 1];
            } else {  // the L1 bucket's own lower bound
                const uint32_t q = b % L.B1r, r = b / L.B1r;
                if (q == 0) { a = 0; c = 0; }
                else {
                    a = L.spl1[2ull * (r * (L.B1r - 1u) + q - 1u)];
                    c = L.spl1[2ull * (r * (L.B1r - 1u) + q - 1u) + 1];
                }
            }
            L.leaf_lb[2 * lid] = a;
            L.leaf_lb[2 * lid + 1] = c;
        }
        if (tid == 0) L.nleaf[b] = B2;
    }
    lds_barrier();
    L2P(5);
    // ---- scatter, staged through LDS: a chunk of W_SC records is counting-sorted by leaf in LDS,
    // then stored so that consecutive threads write consecutive records of one leaf (a run of ~8
    // records per leaf per chunk instead of one 16-byte store per record at a random place: the
    // unstaged scatter wrote 2x its bytes to HBM and ran at a fifth of the read passes' rate)
    constexpr uint32_t WSC = SEG ? W_SCS : W_SC;   // SEG: the top of the stage holds the digit -> leaf map
    constexpr uint32_t SU = WSC / W_WG;
    static_assert(WSC % W_WG == 0, "a chunk is whole records per thread");
    v2 *stg = reinterpret_cast<v2 *>(s_smp);              // the chunk in leaf order (the sample's LDS)
    uint16_t *stl = reinterpret_cast<uint16_t *>(s_spl);  // its leaves (the splitters' LDS)
    GASW v2 *outv = reinterpret_cast<GASW v2 *>(gw(L.out) + 2 * obase);
    if (samp && s_ovf) {   // (uniform: read after the barrier above) capacities past the budget
        if (tid == 0) L.redo_flags[b] = 1u;
        return;
    }
    for (uint64_t c0 = 0; c0 < nb; c0 += WSC) {
        const uint32_t nc = (uint32_t)min<uint64_t>(WSC, nb - c0);
        v2 x[SU];
        uint32_t j[SU], r[SU];
        // SEG: each thread finds its first record's segment by a search over the bucket's segment starts
        // (s_cseg, LDS), then walks forward (its records are W_WG apart; segments hold ~1 K records)
        uint32_t sw = 0;
        if (SEG) {
            const uint64_t q0 = c0 + min(tid, nc - 1u);
            uint32_t lo = 0, hi = L.grid + 1u;  // s_cseg[lo] <= q0 < s_cseg[hi]
            while (hi - lo > 1u) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_cseg[mid] <= q0) lo = mid;
                else hi = mid;
            }
            sw = lo;
        }
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u) {
            const uint32_t p = tid + u * W_WG;
            const uint64_t i = c0 + min(p, nc - 1u);
            if (SEG) {
                while (s_cseg[sw + 1] <= i) ++sw;
                uint64_t a, c;
                seg_load(L, b, sw, i - s_cseg[sw], a, c);
                x[u] = v2{a, c};
            } else {
                x[u] = inv[i];
            }
            // the histogram pass's leaf (no second splitter search); SEG: the digit again from the
            // record (three LDS code reads: cheaper than storing and re-reading a digit per record)
            if (SEG) j[u] = B2 > 1 ? lmap[sub_of(x[u].x, x[u].y)] : 0u;
            else j[u] = gw(L.sub)[base + i];
        }
        if (tid < B2) s_cnt[tid] = 0;
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u)
            if (tid + u * W_WG < nc) r[u] = atomicAdd(&s_cnt[j[u]], 1u);
        lds_barrier();
        {
            uint32_t tot;
            const uint32_t ex = block_scan_excl(tid < B2 ? s_cnt[tid] : 0u, s_ws, &tot);
            if (tid < B2) s_bst[tid] = ex;
        }
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u)
            if (tid + u * W_WG < nc) {
                const uint32_t p = s_bst[j[u]] + r[u];
                stg[p] = x[u];
                stl[p] = (uint16_t)j[u];
            }
        lds_barrier();
#pragma unroll
        for (uint32_t u = 0; u < SU; ++u) {
            const uint32_t p = tid + u * W_WG;
            if (p < nc) {
                const uint32_t q = stl[p];
                const uint32_t d = s_cur[q] + (p - s_bst[q]);
                if (!SEG || d < s_end[q]) outv[d] = stg[p];
                else s_ovf = 1u;   // a sampled leaf past its region: the bucket is redone exactly
            }
        }
        lds_barrier();
        if (tid < B2) s_cur[tid] += s_cnt[tid];   // the thread that zeroes s_cnt[tid] next chunk
    }
    lds_barrier();
    if (samp && s_ovf) {   // a leaf overflowed its region: the bucket is redone exactly
        if (tid == 0) L.redo_flags[b] = 1u;
        return;
    }
    {   // where each leaf ends in `out`, and its first slot in the dense order (exact counts, scanned)
        const uint64_t lid = (uint64_t)b * MRG_WIDE_MAXB2 + tid;
        const uint32_t cnt = tid < B2 ? s_cur[tid] - (uint32_t)(L.leaf_lo[lid] - obase) : 0u;
        uint32_t tot;
        const uint32_t ex = block_scan_excl(cnt, s_ws, &tot);
        if (tid < B2) {
            L.leaf_hi[lid] = obase + s_cur[tid];
            L.leaf_dlo[lid] = base + ex;
        }
    }
    L2P(6);
#ifdef MRG_WIDE_PROF
    if (tid == 0)
        for (int i = 0; i < 7; ++i) atomicAdd(&g_l2prof[i], (unsigned long long)l2acc[i]);
#endif
}
#undef L2P

// ---------------------------------------------------------------- leaves
struct LeafArgs {
    const uint64_t *kin;     // records in leaf order, 2 words each
    uint64_t *kout;          // distinct keys, 2 words each, at slot leaf_out[leaf] + i
    const uint64_t *bstart;
    const uint32_t *nleaf;
    const uint64_t *leaf_lo, *leaf_lb;
    uint32_t B1r, R;
    // weighted keys (flushed map tables, aggregated), sorted by (part, k0, k1)
    const uint64_t *wk0, *wk1, *wcnt;
    const uint32_t *wpart;
    uint64_t nw;
    uint32_t maxd;           // distinct keys a leaf may hold (W_MAXD; test knob smaller)
    // outputs: out key slot = leaf_lo + (weighted keys before the leaf); [slot] counts
    uint64_t *ocnt;
    uint64_t *leaf_out;      // first output slot of each leaf
    uint32_t *leaf_nd;       // distinct keys written (0 for an overflowed leaf)
    uint64_t *leaf_bytes;    // bytes of the leaf's lines "{key} {count}\n"
    uint32_t *leaf_last;     // bytes of its last line
    uint32_t *ovf_list;      // overflowed leaves (ids)
    unsigned long long *ovf_n;
    unsigned long long *nkeys;
    uint64_t *wr;            // [leaves][2] weighted-key range of each leaf (k_wranges)
    unsigned long long *prof;  // MRG_WIDE_PROF builds: phase clocks
    uint32_t *big_list;      // leaves the one-wave kernel passes to the workgroup kernel
    unsigned long long *big_n;
    uint32_t *leaf_pk;       // 1: the leaf's counts sit in the low word of its key slots (no ocnt entry)
    uint32_t pack;           // packing allowed (every count fits 32 bits)
    const uint64_t *leaf_hi;   // one past each leaf's last record in kin (L2 may leave gaps between leaves)
    const uint64_t *leaf_dlo;  // each leaf's first record in the dense order: its output slots start there
};

// first weighted key >= (p, a, b)
__device__ __forceinline__ uint64_t w_lower(const LeafArgs &L, uint32_t p, uint64_t a, uint64_t b) {
    uint64_t lo = 0, hi = L.nw;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const uint32_t mp = L.wpart[mid];
        const bool less = mp < p || (mp == p && key_lt(L.wk0[mid], L.wk1[mid], a, b));
        if (less) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t w_hash(uint64_t a, uint64_t b) {
    return (uint32_t)(mrg_fmix64(a ^ mrg_fmix64(b)) >> 20);
}
__device__ __forceinline__ uint32_t line_len(uint64_t k0, uint64_t k1, uint64_t c) {
    return mrg_short_len(k0, k1) + 2u + mrg_ndigits(c);
}

// weighted-key range [wr[2l], wr[2l+1]) of every leaf l: partition r's keys in [lb_l, lb_{l+1})
__device__ __forceinline__ void leaf_wrange(const LeafArgs &L, uint64_t lid, uint64_t &wlo, uint64_t &whi) {
    const uint32_t b = (uint32_t)(lid / MRG_WIDE_MAXB2), j = (uint32_t)(lid % MRG_WIDE_MAXB2);
    const uint32_t r = b / L.B1r, nl = L.nleaf[b];
    wlo = w_lower(L, r, L.leaf_lb[2 * lid], L.leaf_lb[2 * lid + 1]);
    if (j + 1 < nl) whi = w_lower(L, r, L.leaf_lb[2 * lid + 2], L.leaf_lb[2 * lid + 3]);
    else if ((b + 1) % L.B1r != 0) {  // next L1 bucket of the same partition
        const uint64_t nid = (uint64_t)(b + 1) * MRG_WIDE_MAXB2;
        whi = w_lower(L, r, L.leaf_lb[2 * nid], L.leaf_lb[2 * nid + 1]);
    } else whi = w_lower(L, r + 1u, 0, 0);
}
__global__ void k_wranges(LeafArgs L, uint32_t B1) {
    const uint64_t lid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lid >= (uint64_t)B1 * MRG_WIDE_MAXB2) return;
    const uint32_t b = (uint32_t)(lid / MRG_WIDE_MAXB2), j = (uint32_t)(lid % MRG_WIDE_MAXB2);
    if (j >= L.nleaf[b]) return;
    uint64_t lo = 0, hi = 0;
    if (L.nw) leaf_wrange(L, lid, lo, hi);
    L.wr[2 * lid] = lo;
    L.wr[2 * lid + 1] = hi;
}

// W_DBITS bits of the 128-bit big-endian key (k0:k1) starting at bit hb (0 = most significant)
constexpr uint32_t W_DBITS = 10;
__device__ __forceinline__ uint32_t key_digit(uint64_t k0, uint64_t k1, uint32_t hb) {
    // top 64 bits of (k0:k1) << hb
    const uint64_t t = hb == 0 ? k0 : (hb < 64 ? (k0 << hb) | (k1 >> (64 - hb)) : k1 << (hb - 64));
    return (uint32_t)(t >> (64 - W_DBITS));
}

// One workgroup per L1 bucket walks its leaves.  Per leaf: sum the records per key in an LDS hash
// table, compact the distinct keys, bucket them by the W_DBITS key bits after their common prefix
// (a counting sort), rank each key inside its (small) bucket by comparisons and store it at its
// final position together with its count; the leaf's line bytes are summed on the way.  The next
// leaf's records are loaded while the current one is sorted.  A leaf whose buckets are large (keys
// that agree beyond those bits) is ordered by an LSD radix sort over its varying key bytes instead.
constexpr uint32_t W_NDIG = 1u << W_DBITS;
constexpr uint32_t W_MAXBKT = 64;         // largest bucket ordered by comparisons
constexpr uint32_t W_LR = (W_MAXD + W_LWG - 1) / W_LWG;   // items per thread (3)
constexpr int W_PF = (int)W_LR;           // records per thread prefetched for the next leaf

__global__ __launch_bounds__(W_LWG, 3) void k_wleaf(LeafArgs L) {
    typedef uint64_t v2 __attribute__((ext_vector_type(2)));
    __shared__ v2 s_k[W_SLOTS];               // table keys (k0, k1); k0 == 0 = empty; then bucket order
    __shared__ uint64_t s_c[W_SLOTS];         // table counts
    __shared__ v2 s_kc[W_MAXD];               // distinct keys, compacted
    __shared__ uint64_t s_cc[W_MAXD];         // their counts
    __shared__ uint16_t s_ia[W_MAXD], s_ib[W_MAXD];   // index lists (radix path)
    // digit counts (u32) + starts (u16), or the radix cells (W_LR x W_LNW x 256 u16): 6 KiB
    __shared__ __attribute__((aligned(16))) uint16_t s_x[W_LR * W_LNW * 256];
    __shared__ uint32_t s_ws[W_LNW];
    __shared__ uint32_t s_nd, s_ovf, s_maxb;
    __shared__ uint64_t s_or0, s_or1, s_bytes;
    uint32_t *s_dcnt = reinterpret_cast<uint32_t *>(s_x);   // counting sort: per-digit count
    uint16_t *s_doff = s_x + 2 * W_NDIG;                     // and start
    v2 *s_kb = s_k;                                          // keys in bucket order (table reused)
    static_assert(2 * W_NDIG * 2 + W_NDIG * 2 <= sizeof(s_x), "digit arrays fit the cells");
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t nlist = (uint32_t)*L.big_n;   // leaves passed on by k_wleafw
    const uint64_t lt = mrg_lanemask_lt();
    const GASW v2 *kin = reinterpret_cast<const GASW v2 *>(gw(L.kin));
    unsigned long long wg_keys = 0;   // distinct keys of this workgroup's leaves (thread 0)
#ifdef MRG_WIDE_PROF  // diagnostic build: per-phase clocks of wave 0, summed into L.prof[8]
    uint64_t pacc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tl = clock64();
#define WP(i) { const uint64_t t_ = clock64(); pacc[i] += t_ - tl; tl = t_; }
#else
#define WP(i)
#endif
    auto leaf_at = [&](uint32_t i, uint64_t &lid, uint64_t &lo, uint64_t &hi) {
        lid = L.big_list[i];
        const uint32_t b = (uint32_t)(lid / MRG_WIDE_MAXB2), j = (uint32_t)(lid % MRG_WIDE_MAXB2);
        (void)b; (void)j;
        lo = L.leaf_lo[lid];
        hi = L.leaf_hi[lid];
    };
    // first W_PF * W_LWG records of leaf j into registers (a record past the leaf: a repeat, unused)
    v2 pf[W_PF], pff = v2{0, 0};   // pff: the leaf's first record (the same in every thread)
#pragma unroll
    for (int u = 0; u < W_PF; ++u) pf[u] = v2{0, 0};
    auto prefetch = [&](uint32_t i) {
        if (i >= nlist) return;
        uint64_t lid, lo, hi;
        leaf_at(i, lid, lo, hi);
        if (hi == lo) return;
#pragma unroll
        for (int u = 0; u < W_PF; ++u) pf[u] = kin[lo + min((uint64_t)(tid + u * W_LWG), hi - lo - 1u)];
        pff = kin[lo];
    };
    prefetch(blockIdx.x);
    if (tid == 0) {
        s_or0 = 0;
        s_or1 = 0;
        s_maxb = 0;
        s_bytes = 0;
    }
    for (uint32_t i = tid; i < W_NDIG; i += W_LWG) s_dcnt[i] = 0;
    lds_barrier();
    for (uint32_t i = blockIdx.x; i < nlist; i += gridDim.x) {
        uint64_t lid, mlo, mhi;
        leaf_at(i, lid, mlo, mhi);
        const uint64_t wlo = L.wr[2 * lid], whi = L.wr[2 * lid + 1];
        const uint64_t nm = mhi - mlo, nwk = whi - wlo;
        const uint64_t out0 = L.leaf_dlo[lid] + wlo;
        v2 cur[W_PF];
#pragma unroll
        for (int u = 0; u < W_PF; ++u) cur[u] = pf[u];
        const v2 f = pff;
        prefetch(i + gridDim.x);   // in flight while this leaf is processed
        const uint64_t NT = nm + nwk;
        GASW v2 *ko = reinterpret_cast<GASW v2 *>(gw(L.kout)) + out0;
        GASW uint64_t *co = gw(L.ocnt) + out0;
        if (NT <= L.maxd) {
            // ---- sort-then-combine (no hash table): every record is an item held in registers; the
            // items are bucketed by the W_DBITS key bits after the leaf's common prefix (a counting
            // sort), ranked inside their bucket by comparisons (equal keys by bucket slot), and the runs
            // of equal keys of the sorted leaf are summed into its distinct keys.  s_dcnt is zero and
            // s_or*, s_maxb, s_bytes are 0 on entry (cleared by the previous leaf).
            v2 key[W_LR];
            uint64_t cnt[W_LR];
            uint64_t o0 = 0, o1 = 0;
            // f: one reference key for the whole workgroup (the leaf's first record).  The keys agree
            // on every bit above the first set bit of OR(key ^ f), so the digit taken from there orders
            // them; with f a member that bit is exactly the first one the keys differ on.
#pragma unroll
            for (uint32_t k = 0; k < W_LR; ++k) {
                const uint64_t p = (uint64_t)k * W_LWG + tid;
                cnt[k] = 0;
                key[k] = f;
                if (p < nm) {
                    key[k] = cur[k];
                    cnt[k] = 1;
                } else if (p < NT) {
                    key[k] = v2{L.wk0[wlo + p - nm], L.wk1[wlo + p - nm]};
                    cnt[k] = L.wcnt[wlo + p - nm];
                }
                o0 |= key[k].x ^ f.x;
                o1 |= key[k].y ^ f.y;
            }
            for (int o = 32; o > 0; o >>= 1) {
                o0 |= __shfl_xor(o0, o);
                o1 |= __shfl_xor(o1, o);
            }
            if (lane == 0 && (o0 | o1)) {
                atomicOr((unsigned long long *)&s_or0, (unsigned long long)o0);
                atomicOr((unsigned long long *)&s_or1, (unsigned long long)o1);
            }
            lds_barrier();
            WP(0);
            const uint64_t r0 = s_or0, r1 = s_or1;
            uint32_t hb = r0 ? (uint32_t)__builtin_clzll(r0) : (r1 ? 64u + (uint32_t)__builtin_clzll(r1) : 0u);
            if (hb > 128u - W_DBITS) hb = 128u - W_DBITS;
            uint32_t dg[W_LR], within[W_LR];
#pragma unroll
            for (uint32_t k = 0; k < W_LR; ++k) {
                const uint64_t p = (uint64_t)k * W_LWG + tid;
                dg[k] = 0xFFFFFFFFu;
                if (p < NT) {
                    dg[k] = key_digit(key[k].x, key[k].y, hb);
                    within[k] = atomicAdd(&s_dcnt[dg[k]], 1u);
                }
            }
            lds_barrier();
            {
                constexpr uint32_t PT = W_NDIG / W_LWG;
                uint32_t v[PT], sum = 0, mx = 0;
#pragma unroll
                for (uint32_t x = 0; x < PT; ++x) {
                    v[x] = s_dcnt[tid * PT + x];
                    sum += v[x];
                    mx = max(mx, v[x]);
                }
                if (mx > W_MAXBKT) atomicMax(&s_maxb, mx);
                uint32_t tot;
                uint32_t run = block_scan_excl<W_LNW>(sum, s_ws, &tot);
#pragma unroll
                for (uint32_t x = 0; x < PT; ++x) {
                    s_doff[tid * PT + x] = (uint16_t)run;
                    run += v[x];
                }
            }
            lds_barrier();
            WP(1);
            const bool small = s_maxb == 0;
            if (small) {
#pragma unroll
                for (uint32_t k = 0; k < W_LR; ++k)
                    if (dg[k] != 0xFFFFFFFFu) s_kb[s_doff[dg[k]] + within[k]] = key[k];
                lds_barrier();
#pragma unroll
                for (uint32_t k = 0; k < W_LR; ++k) {
                    if (dg[k] == 0xFFFFFFFFu) continue;
                    const uint32_t bs = s_doff[dg[k]], bn = s_dcnt[dg[k]];
                    uint32_t rank = 0;
                    for (uint32_t q = 0; q < bn; ++q) {
                        const v2 x = s_kb[bs + q];
                        rank += (key_lt(x.x, x.y, key[k].x, key[k].y) ||
                                 (x.x == key[k].x && x.y == key[k].y && q < within[k])) ? 1u : 0u;
                    }
                    s_kc[bs + rank] = key[k];
                    s_cc[bs + rank] = cnt[k];
                }
                lds_barrier();
                WP(2);
                for (uint32_t i = tid; i < W_NDIG; i += W_LWG) s_dcnt[i] = 0;   // for the next leaf
                // runs of equal keys: thread t owns sorted items [W_LR t, W_LR t + W_LR)
                const uint32_t p0 = tid * W_LR;
                bool head[W_LR];
                uint32_t nh = 0;
#pragma unroll
                for (uint32_t k = 0; k < W_LR; ++k) {
                    const uint32_t p = p0 + k;
                    head[k] = false;
                    if (p < NT) {
                        head[k] = p == 0;
                        if (p) {
                            const v2 a = s_kc[p - 1], c = s_kc[p];
                            head[k] = a.x != c.x || a.y != c.y;
                        }
                    }
                    nh += head[k] ? 1u : 0u;
                }
                uint32_t D;
                uint32_t dpos = block_scan_excl<W_LNW>(nh, s_ws, &D);
                WP(3);
                uint64_t bytes = 0;
#pragma unroll
                for (uint32_t k = 0; k < W_LR; ++k) {
                    if (!head[k]) continue;
                    const uint32_t p = p0 + k;
                    const v2 x = s_kc[p];
                    uint64_t n = s_cc[p];
                    for (uint32_t q = p + 1; q < NT; ++q) {
                        const v2 y = s_kc[q];
                        if (y.x != x.x || y.y != x.y) break;
                        n += s_cc[q];
                    }
                    ko[dpos] = x;
                    co[dpos] = n;
                    const uint32_t ll = line_len(x.x, x.y, n);
                    bytes += ll;
                    if (dpos == D - 1) L.leaf_last[lid] = ll;
                    ++dpos;
                }
                for (int o = 32; o > 0; o >>= 1) bytes += __shfl_xor(bytes, o);
                if (lane == 0 && bytes) atomicAdd((unsigned long long *)&s_bytes, (unsigned long long)bytes);
                lds_barrier();
                if (tid == 0) {
                    L.leaf_out[lid] = out0;
                    L.leaf_nd[lid] = D;
                    L.leaf_bytes[lid] = s_bytes;
                    if (D == 0) L.leaf_last[lid] = 0;
                    wg_keys += D;
                    s_or0 = 0;
                    s_or1 = 0;
                    s_bytes = 0;
                }
                lds_barrier();
                WP(4);
                continue;
            }
            // a bucket too large to rank by comparisons (many equal keys): the hash path below, once
            // every wave has read s_maxb
            lds_barrier();
        }
        // table size: a power of two >= 2 x records (a leaf of duplicates still fits: distinct counts)
        uint32_t S = 64;
        while (S < W_SLOTS && (uint64_t)S < 2 * (nm + nwk)) S <<= 1;
        for (uint32_t i = tid; i < S; i += W_LWG) {
            s_k[i] = v2{MRG_EMPTY_K0, MRG_EMPTY_K1};
            s_c[i] = 0;
        }
        if (tid == 0) {
            s_nd = 0;
            s_ovf = 0;
            s_maxb = 0;
            s_or0 = 0;
            s_or1 = 0;
            s_bytes = 0;
        }
        lds_barrier();
        WP(0);
        // ---- sum the records per key (exact: full keys compared; slots fill monotonically)
        auto add = [&](uint64_t a, uint64_t c, uint64_t n) {
            uint32_t slot = w_hash(a, c) & (S - 1u);
            for (uint32_t p = 0; p < S; ++p) {
                const v2 k = s_k[slot];
                if (k.x == a && k.y == c) {
                    atomicAdd((unsigned long long *)&s_c[slot], (unsigned long long)n);
                    return;
                }
                if (k.x == MRG_EMPTY_K0 || (k.x == a && k.y == MRG_EMPTY_K1)) {
                    unsigned long long *kp = reinterpret_cast<unsigned long long *>(&s_k[slot]);
                    const unsigned long long x = atomicCAS(kp, MRG_EMPTY_K0, a);
                    if (x == MRG_EMPTY_K0 || x == a) {
                        const unsigned long long y = atomicCAS(kp + 1, MRG_EMPTY_K1, c);
                        if (y == MRG_EMPTY_K1 || y == c) {
                            // a slot becomes a key exactly once, by the CAS that sets k1
                            if (y == MRG_EMPTY_K1 && atomicAdd(&s_nd, 1u) >= L.maxd) s_ovf = 1;
                            atomicAdd((unsigned long long *)&s_c[slot], (unsigned long long)n);
                            return;
                        }
                    }
                }
                slot = (slot + 1u) & (S - 1u);
            }
            s_ovf = 1;  // no slot left
        };
#pragma unroll
        for (int u = 0; u < W_PF; ++u)
            if ((uint64_t)(tid + u * W_LWG) < nm) add(cur[u].x, cur[u].y, 1ull);
        for (uint64_t i = tid + (uint64_t)W_PF * W_LWG; i < nm; i += W_LWG) {   // beyond the prefetch
            if (s_ovf) break;
            const v2 x = kin[mlo + i];
            add(x.x, x.y, 1ull);
        }
        for (uint64_t i = tid; i < nwk; i += W_LWG) {
            if (s_ovf) break;
            add(L.wk0[wlo + i], L.wk1[wlo + i], L.wcnt[wlo + i]);
        }
        lds_barrier();
        WP(1);
        if (s_ovf) {  // finished by the global fallback (mrgpu.cpp)
            if (tid == 0) {
                const unsigned long long k = atomicAdd(L.ovf_n, 1ull);
                L.ovf_list[k] = (uint32_t)lid;
                L.leaf_out[lid] = out0;
                L.leaf_nd[lid] = 0;
                L.leaf_bytes[lid] = 0;
                L.leaf_last[lid] = 0;
                s_or0 = 0;
                s_or1 = 0;
                s_maxb = 0;
                s_bytes = 0;
            }
            for (uint32_t i = tid; i < W_NDIG; i += W_LWG) s_dcnt[i] = 0;
            lds_barrier();
            continue;
        }
        // ---- compact the distinct keys (s_kc, s_cc); clear the digit counts
        const uint32_t D = s_nd;
        lds_barrier();
        if (tid == 0) s_nd = 0;
        for (uint32_t i = tid; i < W_NDIG; i += W_LWG) s_dcnt[i] = 0;
        lds_barrier();
        for (uint32_t i0 = 0; i0 < S; i0 += W_LWG) {
            const uint32_t i = i0 + tid;
            v2 k = v2{0, 0};
            uint64_t n = 0;
            if (i < S) {
                k = s_k[i];
                n = s_c[i];
            }
            const bool full = k.x != MRG_EMPTY_K0;
            const uint64_t m = __ballot(full);
            uint32_t basew = 0;
            if (lane == 0 && m) basew = atomicAdd(&s_nd, (uint32_t)__popcll(m));
            basew = __shfl(basew, 0);
            if (full) {
                const uint32_t pos = basew + (uint32_t)__popcll(m & lt);
                s_kc[pos] = k;
                s_cc[pos] = n;
            }
        }
        lds_barrier();
        // ---- my items (compacted index p = k * W_LWG + tid) in registers; the bits keys differ on
        const uint32_t NR = (D + W_LWG - 1) / W_LWG;   // items per thread (<= W_LR)
        v2 key[W_LR];
        uint64_t cnt[W_LR];
        {
            const v2 f = D ? s_kc[0] : v2{0, 0};
            uint64_t o0 = 0, o1 = 0;
#pragma unroll
            for (uint32_t k = 0; k < W_LR; ++k) {
                const uint32_t p = k * W_LWG + tid;
                if (k < NR && p < D) {
                    key[k] = s_kc[p];
                    cnt[k] = s_cc[p];
                    o0 |= key[k].x ^ f.x;
                    o1 |= key[k].y ^ f.y;
                }
            }
            for (int o = 32; o > 0; o >>= 1) {
                o0 |= __shfl_xor(o0, o);
                o1 |= __shfl_xor(o1, o);
            }
            if (lane == 0 && (o0 | o1)) {
                atomicOr((unsigned long long *)&s_or0, (unsigned long long)o0);
                atomicOr((unsigned long long *)&s_or1, (unsigned long long)o1);
            }
        }
        lds_barrier();
        WP(2);
        const uint64_t o0 = s_or0, o1 = s_or1;
        // first differing bit (0 = most significant bit of k0); the digit = the W_DBITS bits from there
        uint32_t hb = o0 ? (uint32_t)__builtin_clzll(o0) : (o1 ? 64u + (uint32_t)__builtin_clzll(o1) : 0u);
        if (hb > 128u - W_DBITS) hb = 128u - W_DBITS;
        // ---- counting sort by digit: bucket counts, then starts
        uint32_t dg[W_LR], within[W_LR];
#pragma unroll
        for (uint32_t k = 0; k < W_LR; ++k) {
            const uint32_t p = k * W_LWG + tid;
            dg[k] = 0xFFFFFFFFu;
            if (k < NR && p < D) {
                dg[k] = key_digit(key[k].x, key[k].y, hb);
                within[k] = atomicAdd(&s_dcnt[dg[k]], 1u);  // slot inside the bucket (any order)
            }
        }
        lds_barrier();
        {  // exclusive scan of the digit counts, W_NDIG / W_LWG per thread; note the largest bucket
            constexpr uint32_t PT = W_NDIG / W_LWG;
            uint32_t v[PT], sum = 0, mx = 0;
            for (uint32_t x = 0; x < PT; ++x) {
                v[x] = s_dcnt[tid * PT + x];
                sum += v[x];
                mx = max(mx, v[x]);
            }
            if (mx > W_MAXBKT) atomicMax(&s_maxb, mx);
            uint32_t tot;
            uint32_t run = block_scan_excl<W_LNW>(sum, s_ws, &tot);
            for (uint32_t x = 0; x < PT; ++x) {
                s_doff[tid * PT + x] = (uint16_t)run;
                run += v[x];
            }
        }
        lds_barrier();
        WP(3);
        uint64_t bytes = 0;
        if (s_maxb == 0) {
            // ---- keys in bucket order, then rank = keys of the same bucket that are smaller
#pragma unroll
            for (uint32_t k = 0; k < W_LR; ++k)
                if (dg[k] != 0xFFFFFFFFu) s_kb[s_doff[dg[k]] + within[k]] = key[k];
            lds_barrier();
#pragma unroll
            for (uint32_t k = 0; k < W_LR; ++k) {
                if (dg[k] == 0xFFFFFFFFu) continue;
                const uint32_t bs = s_doff[dg[k]], bn = s_dcnt[dg[k]];
                uint32_t rank = 0;
                uint32_t q = 0;
                for (; q + 2 <= bn; q += 2) {   // two independent LDS reads per step
                    const v2 x = s_kb[bs + q], y = s_kb[bs + q + 1];
                    rank += (key_lt(x.x, x.y, key[k].x, key[k].y) ? 1u : 0u) +
                            (key_lt(y.x, y.y, key[k].x, key[k].y) ? 1u : 0u);
                }
                if (q < bn) {
                    const v2 x = s_kb[bs + q];
                    rank += key_lt(x.x, x.y, key[k].x, key[k].y) ? 1u : 0u;
                }
                const uint32_t pos = bs + rank;
                ko[pos] = key[k];
                co[pos] = cnt[k];
                const uint32_t ll = line_len(key[k].x, key[k].y, cnt[k]);
                bytes += ll;
                if (pos == D - 1) L.leaf_last[lid] = ll;
            }
        } else {
            // ---- LSD radix sort of the index list by the varying key bytes (stable, per-wave ranks)
            for (uint32_t p = tid; p < D; p += W_LWG) s_ia[p] = (uint16_t)p;
            lds_barrier();
            const int qlo = (int)(hb >> 3);
            const int qhi = o1 ? 15 - (int)(__builtin_ctzll(o1) >> 3) : 7 - (int)(__builtin_ctzll(o0) >> 3);
            uint16_t *src = s_ia, *dst = s_ib;
            uint16_t *s_wc = s_x;
            for (int q = qhi; q >= qlo; --q) {
                for (uint32_t i = tid; i < NR * W_LNW * 256; i += W_LWG) s_wc[i] = 0;
                lds_barrier();
                uint32_t rk[W_LR];
#pragma unroll
                for (uint32_t k = 0; k < W_LR; ++k) {
                    if (k >= NR) break;
                    const uint32_t p = k * W_LWG + tid;
                    const bool valid = p < D;
                    uint32_t d = 0;
                    if (valid) {
                        const v2 x = s_kc[src[p]];
                        d = key_byte(x.x, x.y, (uint32_t)q);
                    }
                    uint64_t peers = __ballot(valid);
                    for (int bt = 0; bt < 8; ++bt) {
                        const uint64_t mb = __ballot(valid && ((d >> bt) & 1u));
                        peers &= ((d >> bt) & 1u) ? mb : ~mb;
                    }
                    const uint32_t rank = (uint32_t)__popcll(peers & lt);
                    if (valid && rank == 0) s_wc[(d * NR + k) * W_LNW + wv] = (uint16_t)__popcll(peers);
                    dg[k] = d;
                    rk[k] = valid ? rank : 0xFFFFFFFFu;
                }
                lds_barrier();
                {  // exclusive scan over the cells in (digit, round, wave) order: stable positions
                    const uint32_t C = 256u * NR * W_LNW, per = C / W_LWG;
                    uint32_t v[4 * W_LR];
                    uint32_t sum = 0;
#pragma unroll
                    for (uint32_t x = 0; x < 4 * W_LR; ++x) {
                        v[x] = x < per ? s_wc[tid * per + x] : 0u;
                        sum += v[x];
                    }
                    uint32_t tot;
                    uint32_t run = block_scan_excl<W_LNW>(sum, s_ws, &tot);
#pragma unroll
                    for (uint32_t x = 0; x < 4 * W_LR; ++x) {
                        if (x < per) s_wc[tid * per + x] = (uint16_t)run;
                        run += v[x];
                    }
                }
                lds_barrier();
#pragma unroll
                for (uint32_t k = 0; k < W_LR; ++k) {
                    if (k >= NR) break;
                    const uint32_t p = k * W_LWG + tid;
                    if (rk[k] != 0xFFFFFFFFu) dst[s_wc[(dg[k] * NR + k) * W_LNW + wv] + rk[k]] = src[p];
                }
                lds_barrier();
                uint16_t *tmp = src;
                src = dst;
                dst = tmp;
            }
            for (uint32_t p = tid; p < D; p += W_LWG) {
                const uint32_t i = src[p];
                const v2 x = s_kc[i];
                const uint64_t n = s_cc[i];
                ko[p] = x;
                co[p] = n;
                const uint32_t ll = line_len(x.x, x.y, n);
                bytes += ll;
                if (p == D - 1) L.leaf_last[lid] = ll;
            }
        }
        WP(4);
        for (int o = 32; o > 0; o >>= 1) bytes += __shfl_xor(bytes, o);
        if (lane == 0 && bytes) atomicAdd((unsigned long long *)&s_bytes, (unsigned long long)bytes);
        lds_barrier();
        if (tid == 0) {
            L.leaf_out[lid] = out0;
            L.leaf_nd[lid] = D;
            L.leaf_bytes[lid] = s_bytes;
            if (D == 0) L.leaf_last[lid] = 0;
            wg_keys += D;
            s_or0 = 0;
            s_or1 = 0;
            s_maxb = 0;
            s_bytes = 0;
        }
        for (uint32_t i = tid; i < W_NDIG; i += W_LWG) s_dcnt[i] = 0;
        lds_barrier();
        WP(5);
    }
#ifdef MRG_WIDE_PROF
    if (tid == 0)
        for (int i = 0; i < 6; ++i) atomicAdd(&L.prof[i], (unsigned long long)pacc[i]);
#endif
    // one device-scope add per workgroup (a per-leaf add on one word would serialise ~2.7 M adds)
    if (tid == 0 && wg_keys) atomicAdd(L.nkeys, wg_keys);
}

// ---------------------------------------------------------------- leaves, one wave each
// The common case: a leaf of at most W_VC items (records + weighted keys) is finished by ONE wave,
// wave-synchronously (LDS traffic inside a wave is ordered; no workgroup barrier), so a CU keeps
// eight independent leaves in flight.  Items sit in registers (W_VIPL per lane).
//   digit   the three key bytes from the first byte the leaf's items differ on, each as its rank
//           among the values present in the leaf, in mixed radix scaled to 512 (below)
//   order   counting sort of the items by digit in LDS, then each item's rank inside its (small)
//           bucket by comparisons (equal keys by bucket slot), which also tells the item whether
//           it heads its run of equal keys, and gives a head the run's summed count;
//   runs    the heads in sorted order, each stored at leaf_out + its rank among the heads (stores
//           coalesced).
// Leaves with more items, or with a bucket of more than W_VMAXB items, are listed for k_wleaf.
#ifndef MRG_WIDE_VC
#define MRG_WIDE_VC 384   // one-wave leaf capacity (r05: 448 -> 384 with digit leaves, v54)
#endif
constexpr uint32_t W_VC = MRG_WIDE_VC;
constexpr uint32_t W_VIPL = W_VC / 64;
#ifndef MRG_WIDE_VND
#define MRG_WIDE_VND 384   // (r06 v08, v10: 512 -> 384 digits, the leaf kernel at 4 waves per SIMD: C5 aggregation -1.5 %)
#endif
constexpr uint32_t W_VND = MRG_WIDE_VND;   // digits
static_assert(W_VND % 64 == 0 && W_VND <= 0x10000u, "digit counts: whole wave rows; starts fit the LDS words");
#ifndef MRG_WIDE_L2U
#define MRG_WIDE_L2U 4
#endif
#ifndef MRG_WIDE_ABL
#define MRG_WIDE_ABL 0
#endif
#ifndef MRG_WIDE_VRG
#define MRG_WIDE_VRG 2
#endif
constexpr uint32_t W_VRG = MRG_WIDE_VRG; // rows whose buckets one trip of the rank loop reads
constexpr uint32_t W_VMAXB = 64;
#ifndef MRG_WIDE_VQ
#define MRG_WIDE_VQ 16   // (r05 v55: 4 -> 16, the last round of waves less ragged: C5 +2 %)
#endif
constexpr uint32_t W_VQ = MRG_WIDE_VQ;  // waves (one-wave workgroups) per L1 bucket
constexpr uint32_t W_VPASS = MRG_WIDE_MAXB2 / W_VQ;   // leaves one wave may pass on
// tunables against the arrays they size (r06; the v59 fault was W_VC outgrowing s_ix's code tables):
static_assert(W_VC % 64 == 0 && W_VIPL * 64 == W_VC, "items per lane: W_VC a whole number of wave rows");
static_assert(W_VC <= 0x8000u, "s_ix holds sorted positions below the 0x8000 padding marker");
static_assert(W_VQ * W_VPASS == MRG_WIDE_MAXB2, "the waves of an L1 bucket pass on at most MAXB2 leaves together");
static_assert(W_VRG >= 1 && W_VRG <= W_VIPL, "rank-loop row groups within the lane's rows");

__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}
__device__ __forceinline__ uint32_t first_bit(uint64_t o0, uint64_t o1) {   // 128 if none
    return o0 ? (uint32_t)__builtin_clzll(o0) : (o1 ? 64u + (uint32_t)__builtin_clzll(o1) : 128u);
}
__device__ __forceinline__ uint32_t key_bit(uint64_t k0, uint64_t k1, uint32_t hb) {
    return hb < 64 ? (uint32_t)(k0 >> (63u - hb)) & 1u : (uint32_t)(k1 >> (127u - hb)) & 1u;
}
__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
    for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o);
    return v;
}

#ifndef MRG_WIDE_VWPE
#define MRG_WIDE_VWPE 4   // waves per SIMD the register budget is held to (117 VGPRs, no spill)
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MRG_WIDE_VWPE))) void k_wleafw(LeafArgs L) {
    typedef uint64_t v2 __attribute__((ext_vector_type(2)));
    __shared__ v2 s_kb[W_VC];            // items in digit-bucket order
    __shared__ uint32_t s_cb[W_VC];      // their counts (a leaf with a larger weighted count is passed on)
    __shared__ __attribute__((aligned(16))) uint16_t s_ix[W_VC];   // sorted position -> bucket slot (and the digit code tables)
    static_assert(sizeof(s_ix) >= 3 * 256, "the leaf digit's three 256-byte code tables live in s_ix");
    __shared__ uint32_t s_dc[W_VND + 1]; // digit counts, then (the scan, in place) digit starts + the end
    uint32_t *const s_ds = s_dc;
    static_assert(MRG_WIDE_VWPE < 4 || sizeof(s_kb) + sizeof(s_cb) + sizeof(s_ix) + sizeof(s_dc) <= 160u * 1024u / 16u,
                  "4 one-wave workgroups per SIMD: 16 per CU share its 160 KiB of LDS");
    const uint32_t lane = threadIdx.x;
    const uint32_t b = blockIdx.x / W_VQ, q0 = blockIdx.x % W_VQ;
    const uint32_t nl = L.nleaf[b];
    const uint32_t cap = min(L.maxd, W_VC);
    const uint64_t lt = mrg_lanemask_lt();
    const GASW v2 *kin = reinterpret_cast<const GASW v2 *>(gw(L.kin));
    GASW v2 *kout = reinterpret_cast<GASW v2 *>(gw(L.kout));
    GASW uint64_t *cout = gw(L.ocnt);
    unsigned long long keys = 0;
    // a leaf for the workgroup kernel (rare: one device atomic each; an LDS list of them cost the
    // LDS that a fourth wave per SIMD needs)
    auto pass_on = [&](uint64_t lid) {
        if (lane == 0) L.big_list[atomicAdd(L.big_n, 1ull)] = (uint32_t)lid;
    };
#ifdef MRG_WIDE_PROF  // diagnostic build: phase clocks of every wave, summed into L.prof[8..13]
    uint64_t vacc[6] = {0, 0, 0, 0, 0, 0}, vtl = clock64();
#define VP(i) { const uint64_t t_ = clock64(); vacc[i] += t_ - vtl; vtl = t_; }
#else
#define VP(i)
#endif
    for (uint32_t j = q0; j < nl; j += W_VQ) {
        VP(5);
        const uint64_t lid = (uint64_t)b * MRG_WIDE_MAXB2 + j;
        const uint64_t mlo = L.leaf_lo[lid], mhi = L.leaf_hi[lid];
        const uint64_t wlo = L.wr[2 * lid], whi = L.wr[2 * lid + 1];
        const uint64_t nm = mhi - mlo, NT = nm + (whi - wlo);
        if (NT > cap) {
            pass_on(lid);
#ifdef MRG_WIDE_PROF
            if (lane == 0) atomicAdd(&L.prof[6], 1ull);
#endif
            continue;
        }
        const uint64_t out0 = L.leaf_dlo[lid] + wlo;
        GASW v2 *ko = kout + out0;
        GASW uint64_t *co = cout + out0;
        v2 key[W_VIPL];
        uint64_t cnt[W_VIPL];
#pragma unroll
        for (uint32_t k = 0; k < W_VIPL; ++k) {
            const uint64_t p = (uint64_t)k * 64u + lane;
            key[k] = v2{0, 0};
            cnt[k] = 0;
            if (p < nm) {
                key[k] = kin[mlo + p];
                cnt[k] = 1;
            } else if (p < NT) {
                key[k] = v2{L.wk0[wlo + p - nm], L.wk1[wlo + p - nm]};
                cnt[k] = L.wcnt[wlo + p - nm];
            }
        }
        // run totals are summed in 32-bit LDS words: a leaf whose counts add up to 2^32 or more goes to
        // the workgroup kernel
        uint64_t csum = 0;
#pragma unroll
        for (uint32_t k = 0; k < W_VIPL; ++k) csum += cnt[k];
        for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o);
        bool big = csum > 0xFFFFFFFFull;
        VP(0);
        if (__any(big)) {   // a count beyond the LDS count width: the workgroup kernel
            pass_on(lid);
            continue;
        }
        // Packed leaf: when every key of the leaf is at most 12 bytes (the low word of k1 is zero
        // padding) and counts fit 32 bits, a count is stored in that low word of its key slot and
        // no count array entry is written (the line writer reads 16 bytes per line instead of 24)
        bool pk = false;
        {
            uint32_t lw = 0;
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) lw |= (uint32_t)key[k].y;   // padding items are zero
            pk = L.pack && !__any(lw != 0u);
        }
        const v2 f = v2{__shfl(key[0].x, 0), __shfl(key[0].y, 0)};   // item 0 (a member if NT > 0)
        uint64_t o0 = 0, o1 = 0;
#pragma unroll
        for (uint32_t k = 0; k < W_VIPL; ++k) {
            if ((uint64_t)k * 64u + lane >= NT) key[k] = f;   // padding: f's twin, never stored
            o0 |= key[k].x ^ f.x;
            o1 |= key[k].y ^ f.y;
        }
        o0 = wave_or(o0);
        o1 = wave_or(o1);
        const uint32_t hb = first_bit(o0, o1);
        uint32_t D = 0, my_last = 0xFFFFFFFFu, my_ll = 0;
        uint64_t bytes = 0;
        if (hb == 128u) {   // every item has the same key (or none): one line
            uint64_t n = 0;
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) n += cnt[k];
            for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o);
            if (NT) {
                D = 1;
                my_ll = line_len(f.x, f.y, n);
                if (lane == 0) {
                    if (pk) {
                        ko[0] = v2{f.x, f.y | n};
                    } else {
                        ko[0] = f;
                        co[0] = n;
                    }
                    my_last = 0;
                    bytes = my_ll;
                }
            }
        } else {
            // digit: the key bytes P, P + 1, P + 2 from the first byte the items differ on, each
            // replaced by its rank among the values that byte takes in this leaf (a per-leaf code
            // table in LDS), combined in mixed radix and scaled to W_VND digits (monotone: a
            // multiply by a rounded-down reciprocal and a shift).  The items agree on every byte
            // before P, so the digit orders them.  Text keys use ~36 of a byte's 256 values; dense
            // codes spread a leaf's items over the digits (r04's 8 raw bits after each side's
            // first differing bit held 7.5 items per bucket on letter keys: the rank loop below
            // took 53 % of the wave cycles; simulated for C5 keys, profiles/r05/v47_*).
            const uint32_t P = hb >> 3;
            uint8_t *code = reinterpret_cast<uint8_t *>(s_ix);   // 3 x 256 bytes (s_ix is free until the rank step)
            auto kbyte = [&](const v2 &k, uint32_t j) -> uint32_t {
                return j < 8u ? (uint32_t)(k.x >> (56u - 8u * j)) & 0xFFu
                              : (j < 16u ? (uint32_t)(k.y >> (56u - 8u * (j - 8u))) & 0xFFu : 0u);
            };
            for (uint32_t i = lane; i < 3u * 64u; i += 64) reinterpret_cast<uint32_t *>(code)[i] = 0;
            wave_lds_sync();
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) {
                if ((uint64_t)k * 64u + lane >= NT) continue;
#pragma unroll
                for (uint32_t t = 0; t < 3; ++t) code[256u * t + kbyte(key[k], P + t)] = 1;
            }
            wave_lds_sync();
            uint32_t nv[3];
#pragma unroll
            for (uint32_t t = 0; t < 3; ++t) {   // presence -> rank among the present values
                uint32_t *cw = reinterpret_cast<uint32_t *>(code + 256u * t);
                const uint32_t w = cw[lane];
                const uint32_t c = (w & 1u) + ((w >> 8) & 1u) + ((w >> 16) & 1u) + (w >> 24);
                const uint32_t inc = wave_scan_incl(c);
                uint32_t r = inc - c, o = 0;
#pragma unroll
                for (uint32_t bb = 0; bb < 4; ++bb) {
                    o |= r << (8u * bb);
                    r += (w >> (8u * bb)) & 1u;
                }
                cw[lane] = o;
                nv[t] = (uint32_t)__shfl(inc, 63);
            }
            const uint32_t N = nv[0] * nv[1] * nv[2];
            const uint64_t Mr = N > W_VND ? ((uint64_t)W_VND << 32) / N : (1ull << 32);
            wave_lds_sync();
            uint32_t dgv[W_VIPL];
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) {
                const uint32_t c0 = code[kbyte(key[k], P)], c1 = code[256u + kbyte(key[k], P + 1u)],
                               c2 = code[512u + kbyte(key[k], P + 2u)];
                const uint32_t x = (c0 * nv[1] + c1) * nv[2] + c2;
                dgv[k] = (uint32_t)(((uint64_t)x * Mr) >> 32);
            }
            for (uint32_t i = lane; i < W_VND; i += 64) s_dc[i] = 0;
            VP(1);
            wave_lds_sync();
            uint32_t dg[W_VIPL], wi[W_VIPL];
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) {
                dg[k] = 0xFFFFFFFFu;
                wi[k] = 0;
                if ((uint64_t)k * 64u + lane < NT) {
                    dg[k] = dgv[k];
                    wi[k] = atomicAdd(&s_dc[dg[k]], 1u);
                }
            }
            wave_lds_sync();
            uint32_t mx = 0;
            {
                constexpr uint32_t PT = W_VND / 64;
                uint32_t v[PT], sum = 0;
#pragma unroll
                for (uint32_t x = 0; x < PT; ++x) {
                    v[x] = s_dc[lane * PT + x];
                    sum += v[x];
                    mx = max(mx, v[x]);
                }
                uint32_t run = wave_scan_incl(sum) - sum;
#pragma unroll
                for (uint32_t x = 0; x < PT; ++x) {
                    s_ds[lane * PT + x] = run;   // (in place: this lane read its counts above)
                    run += v[x];
                }
                if (lane == 63) s_ds[W_VND] = run;
                for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o));
#ifdef MRG_WIDE_PROF
                uint32_t nz = 0;
#pragma unroll
                for (uint32_t x = 0; x < PT; ++x) nz += v[x] != 0u ? 1u : 0u;
                for (int o = 32; o > 0; o >>= 1) nz += (uint32_t)__shfl_xor(nz, o);
                if (lane == 0) {
                    atomicAdd(&L.prof[14], (unsigned long long)nz);
                    atomicAdd(&L.prof[15], (unsigned long long)mx);
                }
#endif
            }
            if (mx > W_VMAXB) {   // many equal (or near-equal) keys: the workgroup kernel
                pass_on(lid);
#ifdef MRG_WIDE_PROF
                if (lane == 0) atomicAdd(&L.prof[7], 1ull);
#endif
                wave_lds_sync();
                continue;
            }
            wave_lds_sync();
            VP(2);
            uint32_t slot[W_VIPL];
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) {
                slot[k] = 0;
                if (dg[k] == 0xFFFFFFFFu) continue;
                slot[k] = s_ds[dg[k]] + wi[k];
                s_kb[slot[k]] = key[k];
                s_cb[slot[k]] = (uint32_t)cnt[k];
            }
            wave_lds_sync();
            // rank inside the bucket by comparisons (equal keys by bucket slot); an item with an equal
            // key in an earlier slot is not its run's head (flag 0x8000 in s_ix); a head with equal
            // keys after it stores the run's summed count in its own s_cb slot (the other members
            // never write, and what they read is unused)
            // every row's bucket walked in one loop (trip q reads position q of all W_VIPL buckets: one
            // LDS wait per trip instead of one per row and position)
            // rank: the items of the bucket before this one, equal keys ordered by bucket slot; fq = the
            // first slot (in the bucket) holding this item's key, so the item heads its run iff fq == wi.
            // A run's other members add their counts to the head's count slot afterwards (an LDS
            // atomic, rare).  Per-row state stays in VGPRs: bool arrays here became SGPR lane masks in
            // a kernel already at the SGPR limit, and their spills cost more than the loop.
            uint32_t bs[W_VIPL], bn[W_VIPL], rank[W_VIPL], fq[W_VIPL];
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) {
                const bool v = dg[k] != 0xFFFFFFFFu;
                bs[k] = v ? s_ds[dg[k]] : 0u;
                bn[k] = v ? s_ds[dg[k] + 1u] - bs[k] : 0u;
                rank[k] = 0;
                fq[k] = wi[k];
            }
#pragma unroll
            for (uint32_t g0 = 0; g0 < W_VIPL; g0 += W_VRG) {
            uint32_t gmax = 0;
#pragma unroll
            for (uint32_t k = g0; k < g0 + W_VRG && k < W_VIPL; ++k) gmax = max(gmax, bn[k]);
#if MRG_WIDE_ABL & 1   // timing only: no rank loop
            gmax = 0;
#endif
            for (uint32_t q = 0; __any(q < gmax); ++q) {
                v2 x[W_VRG];
#pragma unroll
                for (uint32_t k = g0; k < g0 + W_VRG && k < W_VIPL; ++k) x[k - g0] = s_kb[min(bs[k] + q, W_VC - 1u)];
#pragma unroll
                for (uint32_t kk = 0; kk < W_VRG; ++kk) {
                    const uint32_t k = g0 + kk;
                    if (k >= W_VIPL || q >= bn[k]) continue;
                    const bool eq = x[kk].x == key[k].x && x[kk].y == key[k].y;
                    const bool before = key_lt(x[kk].x, x[kk].y, key[k].x, key[k].y) || (eq && q < wi[k]);
                    rank[k] += before ? 1u : 0u;
                    fq[k] = (eq && q < fq[k]) ? q : fq[k];
                }
            }
            }
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) {
                if (dg[k] == 0xFFFFFFFFu) continue;
                const bool member = fq[k] != wi[k];
                s_ix[bs[k] + rank[k]] = (uint16_t)(slot[k] | (member ? 0x8000u : 0u));
                if (member) atomicAdd(&s_cb[bs[k] + fq[k]], (uint32_t)cnt[k]);
            }
            wave_lds_sync();
            VP(3);
            // the heads in sorted order (position p = k * 64 + lane): each is one distinct key, stored
            // at its rank among the heads
            uint32_t e[W_VIPL];
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) e[k] = k * 64u + lane < NT ? s_ix[k * 64u + lane] : 0x8000u;
            v2 xs[W_VIPL];
            uint32_t cs[W_VIPL];
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) {
                xs[k] = s_kb[e[k] & 0x7FFFu];
                cs[k] = s_cb[e[k] & 0x7FFFu];
            }
#pragma unroll
            for (uint32_t k = 0; k < W_VIPL; ++k) {
                const bool head = (e[k] & 0x8000u) == 0u;
                const uint64_t hm = __ballot(head);
                if (head) {
                    const uint32_t dpos = D + (uint32_t)__popcll(hm & lt);
                    const v2 x = xs[k];
                    const uint64_t n = cs[k];
                    if (pk) {
                        ko[dpos] = v2{x.x, x.y | n};
                    } else {
                        ko[dpos] = x;
                        co[dpos] = n;
                    }
                    my_ll = line_len(x.x, x.y, n);
                    bytes += my_ll;
                    my_last = dpos;
                }
                D += (uint32_t)__popcll(hm);
            }
        }
        VP(4);
        if (D && my_last == D - 1) L.leaf_last[lid] = my_ll;
        for (int o = 32; o > 0; o >>= 1) bytes += __shfl_xor(bytes, o);
        if (lane == 0) {
            L.leaf_out[lid] = out0;
            L.leaf_nd[lid] = D;
            L.leaf_bytes[lid] = bytes;
            L.leaf_pk[lid] = pk ? 1u : 0u;
            if (D == 0) L.leaf_last[lid] = 0;
        }
        keys += D;
        wave_lds_sync();
    }
#ifdef MRG_WIDE_PROF
    if (lane == 0)
        for (int i = 0; i < 6; ++i) atomicAdd(&L.prof[8 + i], (unsigned long long)vacc[i]);
#endif
#undef VP
    if (lane == 0 && keys) atomicAdd(L.nkeys, keys);
}

// last-group drop (worker.rs:169-184): the last key of the last non-empty leaf of partition r
__global__ void k_wdrop(const uint32_t *nleaf, uint32_t B1r, uint32_t R, const uint32_t *leaf_nd,
                        uint64_t *leaf_bytes, const uint32_t *leaf_last, uint32_t *leaf_drop) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    for (int q = (int)B1r - 1; q >= 0; --q) {
        const uint32_t b = r * B1r + (uint32_t)q;
        for (int j = (int)nleaf[b] - 1; j >= 0; --j) {
            const uint64_t lid = (uint64_t)b * MRG_WIDE_MAXB2 + (uint32_t)j;
            if (leaf_nd[lid]) {
                leaf_bytes[lid] -= leaf_last[lid];
                leaf_drop[lid] = 1;
                return;
            }
        }
    }
}

// ---------------------------------------------------------------- lines
// One workgroup per L1 bucket streams the bucket's distinct keys (all its leaves, the dropped last
// key of a partition excluded) in chunks of W_WCH, one key per thread: key i of the bucket -> its
// leaf by a search of the leaves' running key counts (LDS), the line built in registers as
// little-endian words, OR-ed into a zeroed LDS stage at its offset from a block scan of the line
// lengths (whole dwords: the first and last are shared with the neighbour lines), then the stage
// is stored as aligned dwords (byte stores only at the two ends of a chunk) and zeroed on the way.
// 512-thread workgroups, several per CU: while one formats, the others load and store.
#ifndef MRG_WIDE_WWAVE
#define MRG_WIDE_WWAVE 1   // 1: one wave per leaf (k_wwritew, r06: C5 format -23 %), 0: one workgroup per L1 bucket (k_wwrite)
#endif
#ifndef MRG_WIDE_WST
#define MRG_WIDE_WST 1   // r06: the stage stored as 16-byte vectors (was dwords)
#endif
constexpr uint32_t W_WWG = 512;
constexpr uint32_t W_WCH = W_WWG;             // keys per chunk
constexpr uint32_t W_STAGE = 40 * W_WCH;      // >= W_WCH lines of <= 16 + 1 + 20 + 1 bytes (+ 3 of shift)

__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// "key count\n" of a short key as little-endian bytes in w[0..4]; returns its length
__device__ __forceinline__ uint32_t line_words(uint64_t k0, uint64_t k1, uint64_t n, uint64_t w[5]) {
    const uint32_t L = mrg_short_len(k0, k1), nd = mrg_ndigits(n);
    // suffix bytes: ' ', the nd digits, '\n' -- little-endian in t0..t2 (at most 22 bytes)
    uint64_t t0 = ' ', t1 = 0, t2 = 0;
    auto put = [&](uint32_t pos, uint64_t byte) {
        const uint64_t v = byte << (8u * (pos & 7u));
        if (pos < 8u) t0 |= v;
        else if (pos < 16u) t1 |= v;
        else t2 |= v;
    };
    if (n < 10u) {
        t0 |= ((uint64_t)('0' + n) << 8) | ((uint64_t)'\n' << 16);
    } else {
        uint64_t v = n;
        for (uint32_t i = nd; i >= 1u; --i) {
            uint32_t dgt;
            if (v <= 0xFFFFFFFFull) {
                const uint32_t v32 = (uint32_t)v;
                dgt = v32 % 10u;
                v = v32 / 10u;
            } else {
                dgt = (uint32_t)(v % 10u);
                v /= 10u;
            }
            put(i, '0' + dgt);
        }
        put(nd + 1u, '\n');
    }
    // key bytes first (big-endian packed -> byte-swapped words), the suffix shifted in at byte L
    w[0] = bswap64(k0);
    w[1] = bswap64(k1);
    const uint32_t q = L >> 3, r = 8u * (L & 7u);
    const uint64_t u0 = t0 << r;
    const uint64_t u1 = (t1 << r) | (r ? t0 >> (64u - r) : 0ull);
    const uint64_t u2 = (t2 << r) | (r ? t1 >> (64u - r) : 0ull);
    const uint64_t u3 = r ? t2 >> (64u - r) : 0ull;
    w[0] |= q == 0u ? u0 : 0ull;
    w[1] |= q == 0u ? u1 : (q == 1u ? u0 : 0ull);
    w[2] = q == 0u ? u2 : (q == 1u ? u1 : u0);
    w[3] = q == 0u ? u3 : (q == 1u ? u2 : u1);
    w[4] = q == 0u ? 0ull : (q == 1u ? u3 : u2);
    return L + 2u + nd;
}

__global__ __launch_bounds__(W_WWG) void k_wwrite(const uint64_t *keys, const uint64_t *ocnt, const uint32_t *leaf_pk,
                                                    const uint32_t *nleaf, const uint64_t *leaf_out,
                                                    const uint32_t *leaf_nd, const uint32_t *leaf_drop,
                                                    const uint64_t *leaf_off, uint8_t *out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_buf[W_STAGE / 4];
    static_assert(W_STAGE >= 15 + 38 * W_WCH + 4 * 11, "a chunk's lines (<= 38 bytes each) at a 0..15-byte stage shift");
    __shared__ uint32_t s_kst[MRG_WIDE_MAXB2 + 1];   // keys before leaf l (this bucket)
    __shared__ uint64_t s_lout[MRG_WIDE_MAXB2];      // first key slot of leaf l; bit 63: counts packed
    __shared__ uint32_t s_ws[W_WWG / 64];
    const uint8_t *sb = reinterpret_cast<const uint8_t *>(s_buf);
    const uint32_t tid = threadIdx.x, b = blockIdx.x;
    const uint32_t nl = nleaf[b];
    const uint64_t l0 = (uint64_t)b * MRG_WIDE_MAXB2;
    for (uint32_t i = tid; i < W_STAGE / 4; i += W_WWG) s_buf[i] = 0;
    {  // running key counts of the leaves (MAXB2 / W_WWG per thread)
        constexpr uint32_t PT = MRG_WIDE_MAXB2 / W_WWG;
        uint32_t v[PT], sum = 0;
        for (uint32_t x = 0; x < PT; ++x) {
            const uint32_t l = tid * PT + x;
            v[x] = l < nl ? leaf_nd[l0 + l] - (leaf_drop[l0 + l] ? 1u : 0u) : 0u;
            if (l < nl) s_lout[l] = leaf_out[l0 + l] | ((uint64_t)(leaf_pk[l0 + l] != 0u) << 63);
            sum += v[x];
        }
        uint32_t tot;
        uint32_t run = block_scan_excl<W_WWG / 64>(sum, s_ws, &tot);
        for (uint32_t x = 0; x < PT; ++x) {
            s_kst[tid * PT + x] = run;
            run += v[x];
        }
        if (tid == 0) s_kst[MRG_WIDE_MAXB2] = tot;
    }
    lds_barrier();
    const uint32_t K = s_kst[MRG_WIDE_MAXB2];
    uint64_t dst = leaf_off[l0];
    // this thread's key of chunk c0: leaf by a search of the running counts, then the key and count
    // loads.  The next chunk's are fetched before this chunk is laid out and stored, so their leaf
    // search and load latency overlap the current chunk's work.
    struct One {
        uint64_t a, c, n;
    };
    // leaf l of key i: s_kst[l] <= i < s_kst[l + 1] (the last such l).  A thread's keys only move
    // forward (by W_WCH per chunk), so its leaf is found by a forward walk from its previous one:
    // about two LDS reads per chunk for leaves of ~250 keys (a binary search over the bucket's up to
    // 1024 leaves was ten dependent reads per key)
    uint32_t lcur = 0;
    auto fetch = [&](uint32_t c0, One &F) {
        const uint32_t i = c0 + tid;
        F.a = F.c = F.n = 0;
        if (i < K) {
            uint32_t lo = lcur;
            while (lo + 1u < nl && s_kst[lo + 1u] <= i) ++lo;
            lcur = lo;
            const uint64_t lo_out = s_lout[lo];
            const uint64_t slot = (lo_out & ~(1ull << 63)) + (i - s_kst[lo]);
            F.a = keys[2 * slot];
            F.c = keys[2 * slot + 1];
            if (lo_out >> 63) {   // packed leaf: the count is the low word of k1
                F.n = F.c & 0xFFFFFFFFull;
                F.c &= ~0xFFFFFFFFull;
            } else {
                F.n = ocnt[slot];
            }
        }
    };
    One cur, nxt;
    if (K) fetch(0, cur);
    for (uint32_t c0 = 0; c0 < K; c0 += W_WCH) {
        if (c0 + W_WCH < K) fetch(c0 + W_WCH, nxt);
        uint64_t w[5];
        const uint32_t ll = c0 + tid < K ? line_words(cur.a, cur.c, cur.n, w) : 0u;
        uint32_t tot;
        const uint32_t at = block_scan_excl<W_WWG / 64>(ll, s_ws, &tot);
        // stage at the output's offset in its 16-byte (MRG_WIDE_WST; else 4-byte) unit: output vectors align in LDS
        const uint32_t sh = (uint32_t)(dst & (MRG_WIDE_WST ? 15u : 3u));
        if (ll) {
            const uint32_t o = sh + at, base = o >> 2, bs = 8u * (o & 3u);
            const uint32_t ndw = ((o & 3u) + ll + 3u) >> 2;
            uint32_t prev = 0;
#pragma unroll
            for (uint32_t j = 0; j < 10; ++j) {
                const uint32_t d = (uint32_t)(w[j >> 1] >> (32u * (j & 1u)));
                const uint32_t e = (d << bs) | (bs ? prev >> (32u - bs) : 0u);
                prev = d;
                if (j < ndw) atomicOr(&s_buf[base + j], e);
            }
            if (10u < ndw) atomicOr(&s_buf[base + 10u], prev >> (32u - bs));
        }
        lds_barrier();
        const uint64_t end = dst + tot;
#if MRG_WIDE_WST
        // whole 16-byte vectors (one dwordx4 store per lane: a 1 KiB wave store), bytes at the two ends
        const uint64_t a16 = (dst + 15u) & ~15ull, e16 = end & ~15ull;
        for (uint64_t x = dst + tid; x < min(a16, end); x += W_WWG) out[x] = sb[sh + (x - dst)];
        for (uint64_t x = max(e16, a16) + tid; x < end; x += W_WWG) out[x] = sb[sh + (x - dst)];
        for (uint64_t v = a16 / 16 + tid; v < e16 / 16; v += W_WWG) {
            const uint32_t i = (sh + (uint32_t)(v * 16 - dst)) / 16;
            reinterpret_cast<uint4 *>(out)[v] = reinterpret_cast<const uint4 *>(s_buf)[i];
        }
#else
        const uint64_t a4 = (dst + 3u) & ~3ull, e4 = end & ~3ull;
        for (uint64_t x = dst + tid; x < min(a4, end); x += W_WWG) out[x] = sb[sh + (x - dst)];
        for (uint64_t x = max(e4, a4) + tid; x < end; x += W_WWG) out[x] = sb[sh + (x - dst)];
        for (uint64_t w4 = a4 / 4 + tid; w4 < e4 / 4; w4 += W_WWG) {
            const uint32_t i = (sh + (uint32_t)(w4 * 4 - dst)) / 4;
            reinterpret_cast<uint32_t *>(out)[w4] = s_buf[i];
        }
#endif
        lds_barrier();
        // zero what this chunk used (its byte-stored ends included) for the next chunk's ORs
        for (uint32_t i = tid; i < (sh + tot + 3u) / 4u; i += W_WWG) s_buf[i] = 0;
        dst = end;
        lds_barrier();
        cur = nxt;
    }
}

// r06: the same lines, one WAVE per leaf and no workgroup barrier.  A leaf's text starts at
// leaf_off[leaf] (the scan of the leaves' line bytes after the drop), so waves write their leaves
// independently: 64 keys per step, line lengths by a wave scan, the lines OR-ed into the wave's own LDS
// stage, whole 16-byte vectors stored, the partial last vector carried to the next step at the
// stage's start; bytes only at the leaf's two ends (the vectors it shares with its neighbours).
constexpr uint32_t WW_WG = 256, WW_NW = WW_WG / 64;
constexpr uint32_t WW_PER = 16;                          // workgroups per L1 bucket (64 waves stride its leaves)
constexpr uint32_t WW_STGW = (16 + 64 * 38 + 64) / 4;   // stage dwords per wave: carried vector + 64 lines + slack
__device__ __forceinline__ void ww_sync() {   // the wave's LDS ops so far have completed (atomics included)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}
__global__ __launch_bounds__(WW_WG) void k_wwritew(const uint64_t *keys, const uint64_t *ocnt, const uint32_t *leaf_pk,
                                                  const uint32_t *nleaf, const uint64_t *leaf_out,
                                                  const uint32_t *leaf_nd, const uint32_t *leaf_drop,
                                                  const uint64_t *leaf_off, uint8_t *out) {
    __shared__ __attribute__((aligned(16))) uint32_t s_stg[WW_NW][WW_STGW];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t b = blockIdx.x / WW_PER, g = (blockIdx.x % WW_PER) * WW_NW + wv;
    const uint32_t nl = nleaf[b];
    uint32_t *stg = s_stg[wv];
    const uint8_t *sb = reinterpret_cast<const uint8_t *>(stg);
    for (uint32_t i = lane; i < WW_STGW; i += 64u) stg[i] = 0;
    ww_sync();
    typedef uint64_t v2 __attribute__((ext_vector_type(2)));
    const v2 *kv = reinterpret_cast<const v2 *>(keys);
    for (uint32_t j = g; j < nl; j += WW_PER * WW_NW) {
        const uint64_t lid = (uint64_t)b * MRG_WIDE_MAXB2 + j;
        const uint32_t K = leaf_nd[lid] - (leaf_drop[lid] ? 1u : 0u);
        if (K == 0u) continue;
        const uint64_t o0 = leaf_out[lid];
        const bool pk = leaf_pk[lid] != 0u;
        const uint64_t lstart = leaf_off[lid];
        uint64_t dst = lstart;                 // next output byte; the stage holds [dst - sh, ...)
        uint32_t sh = (uint32_t)(dst & 15u);
        for (uint32_t c0 = 0; c0 < K; c0 += 64u) {
            // every lane formats a line (inactive lanes the leaf's first key, then ll = 0): an earlier
            // version with the load and format inside `if (i < K)` wrote a stray 0x83 into 1 % of the
            // lines (the compiled divergent block; found by byte comparison with k_wwrite, tools/dbg_ww.py)
            const uint32_t i = c0 + lane;
            const bool act = i < K;
            const uint64_t slot = o0 + (act ? i : 0u);
            const v2 kk = kv[slot];
            const uint64_t nw = pk ? (kk.y & 0xFFFFFFFFull) : ocnt[slot];
            const uint64_t c = pk ? (kk.y & ~0xFFFFFFFFull) : kk.y;
            uint64_t w[5] = {0, 0, 0, 0, 0};
            const uint32_t lw = line_words(kk.x, c, nw, w);
            const uint32_t ll = act ? lw : 0u;
            const uint32_t incl = wave_scan_incl(ll), tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            if (ll) {
                const uint32_t o = sh + incl - ll, base = o >> 2, bs = 8u * (o & 3u);
                const uint32_t ndw = ((o & 3u) + ll + 3u) >> 2;
                uint32_t prev = 0;
#pragma unroll
                for (uint32_t x = 0; x < 10; ++x) {
                    const uint32_t d = (uint32_t)(w[x >> 1] >> (32u * (x & 1u)));
                    const uint32_t e = (d << bs) | (bs ? prev >> (32u - bs) : 0u);
                    prev = d;
                    if (x < ndw) atomicOr(&stg[base + x], e);
                }
                if (10u < ndw) atomicOr(&stg[base + 10u], prev >> (32u - bs));
            }
            ww_sync();
            const uint64_t end = dst + tot, vb = dst - sh;   // stage byte 0 = output byte vb (16-aligned)
            const bool last = c0 + 64u >= K;
            const uint32_t nfull = (uint32_t)((end - vb) >> 4);   // whole vectors of the stage
            // vector 0 of the leaf's first step holds the previous leaf's last bytes: bytes from lstart on
            if (c0 == 0u && sh != 0u) {
                const uint32_t e0 = (uint32_t)min<uint64_t>(16u, end - vb);
                if (lane >= sh && lane < e0) out[vb + lane] = sb[lane];
            }
            for (uint32_t v = lane; v < nfull; v += 64u)
                if (v != 0u || c0 != 0u || sh == 0u)
                    reinterpret_cast<uint4 *>(out + vb)[v] = reinterpret_cast<const uint4 *>(stg)[v];
            const uint32_t rem = (uint32_t)(end - vb) & 15u;   // bytes of the partial last vector
            if (last) {   // the leaf's last bytes (shared with the next leaf's first vector)
                if (lane < rem && !(nfull == 0u && c0 == 0u && vb + lane < lstart)) out[vb + 16u * nfull + lane] = sb[16u * nfull + lane];
            }
            ww_sync();
            // carry the partial vector to the stage's start (or clear it after the leaf) and zero the rest
            uint32_t cv = 0;
            if (lane < 4u) cv = stg[4u * nfull + lane];
            const uint32_t used = (16u * nfull + rem + 3u) >> 2;
            ww_sync();
            for (uint32_t x = lane; x < used; x += 64u) stg[x] = 0;
            ww_sync();
            if (!last && lane < 4u) stg[lane] = cv;
            ww_sync();
            dst = end;
            sh = rem;
        }
    }
}

// part_off[r] = byte offset of partition r's first leaf; part_off[R] = total
__global__ void k_wpart_off(const uint64_t *leaf_off, uint32_t B1r, uint32_t R, uint64_t total, uint64_t *part_off) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < R) part_off[r] = leaf_off[(uint64_t)r * B1r * MRG_WIDE_MAXB2];
    else if (r == R) part_off[r] = total;
}

// dense KeySet (for consumers other than the line writer): leaf l's keys go to dense_off[l] ..
__global__ __launch_bounds__(256) void k_wdense(const uint64_t *keys, const uint64_t *ocnt, const uint32_t *leaf_pk,
                                                const uint64_t *leaf_out, const uint32_t *leaf_nd,
                                                const uint32_t *dense_off, uint32_t B1r, KeySet ks) {
    const uint64_t lid = blockIdx.x;
    const uint32_t D = leaf_nd[lid];
    const uint64_t o0 = leaf_out[lid], d0 = dense_off[lid];
    const bool pk = leaf_pk[lid] != 0u;
    const uint32_t part = (uint32_t)(lid / MRG_WIDE_MAXB2) / B1r;
    for (uint32_t p = threadIdx.x; p < D; p += blockDim.x) {
        const uint64_t a = keys[2 * (o0 + p)], cw = keys[2 * (o0 + p) + 1];
        const uint64_t c = pk ? cw & ~0xFFFFFFFFull : cw;
        ks.k0[d0 + p] = a;
        ks.k1[d0 + p] = c;
        ks.cnt[d0 + p] = pk ? (cw & 0xFFFFFFFFull) : ocnt[o0 + p];
        ks.len[d0 + p] = mrg_short_len(a, c);
        ks.part[d0 + p] = part;
        ks.doc[d0 + p] = MRG_EMPTY_DOC;
        ks.hoff[d0 + p] = MRG_NO_HEAP;
    }
}

// ---------------------------------------------------------------- overflowed leaves: global sort
// records of the listed leaves -> SortRec{key, part = list position, idx = count slot}, counts apart
__global__ void k_wfb_count(const uint32_t *list, uint32_t nlist, const uint64_t *leaf_lo, const uint64_t *leaf_hi,
                            const uint64_t *wrange, uint64_t *cnt) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nlist) return;
    const uint64_t lid = list[k];
    const uint64_t mlo = leaf_lo[lid], mhi = leaf_hi[lid];
    cnt[k] = (mhi - mlo) + (wrange[2 * k + 1] - wrange[2 * k]);
}
__global__ void k_wfb_gather(const uint32_t *list, const uint64_t *off, const uint64_t *leaf_lo, const uint64_t *leaf_hi,
                             const uint64_t *wrange, const uint64_t *kin, const uint64_t *wk0,
                             const uint64_t *wk1, const uint64_t *wcnt, SortRec *recs, uint64_t *rcnt) {
    const uint32_t k = blockIdx.x;
    const uint64_t lid = list[k];
    const uint64_t mlo = leaf_lo[lid], mhi = leaf_hi[lid];
    const uint64_t wlo = wrange[2 * k], whi = wrange[2 * k + 1];
    const uint64_t nm = mhi - mlo, n = nm + (whi - wlo), o = off[k];
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        SortRec r;
        uint64_t c;
        if (i < nm) {
            r.k0 = kin[2 * (mlo + i)];
            r.k1 = kin[2 * (mlo + i) + 1];
            c = 1;
        } else {
            r.k0 = wk0[wlo + i - nm];
            r.k1 = wk1[wlo + i - nm];
            c = wcnt[wlo + i - nm];
        }
        r.part = k;
        r.doc = 0;
        r.idx = (uint32_t)(o + i);
        r.pad = 0;
        recs[o + i] = r;
        rcnt[o + i] = c;
    }
}
// the leaf weighted ranges of the listed leaves (computed by k_wranges)
__global__ void k_wfb_wrange(LeafArgs L, const uint32_t *list, uint32_t nlist, uint64_t *wrange) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nlist) return;
    const uint64_t lid = list[k];
    wrange[2 * k] = L.wr[2 * lid];
    wrange[2 * k + 1] = L.wr[2 * lid + 1];
}
// sorted records -> run heads (new key or new leaf)
__global__ void k_wfb_heads(const SortRec *r, uint64_t n, uint64_t *head) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    head[i] = (i == 0 || r[i].part != r[i - 1].part || r[i].k0 != r[i - 1].k0 || r[i].k1 != r[i - 1].k1) ? 1u : 0u;
}
// run heads write their key + summed count at the leaf's next output slot; E = scan of heads,
// lfirst[k] = run index of list leaf k's first run
__global__ void k_wfb_emit(const SortRec *r, uint64_t n, const uint64_t *head, const uint64_t *E, const uint64_t *rcnt,
                           const uint32_t *list, const uint64_t *lfirst, const uint64_t *leaf_out, uint64_t *keys,
                           uint64_t *ocnt) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !head[i]) return;
    uint64_t c = 0, e = i;
    do {
        c += rcnt[r[e].idx];
        ++e;
    } while (e < n && !head[e]);
    const uint32_t k = r[i].part;
    const uint64_t slot = leaf_out[list[k]] + (E[i] - lfirst[k]);
    keys[2 * slot] = r[i].k0;
    keys[2 * slot + 1] = r[i].k1;
    ocnt[slot] = c;
}
__global__ void k_wfb_lfirst(const SortRec *r, uint64_t n, const uint64_t *head, const uint64_t *E, uint64_t *lfirst) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == 0 || r[i].part != r[i - 1].part) lfirst[r[i].part] = E[i];
}
// stats of the finished leaves: distinct keys, bytes, last line
__global__ void k_wfb_stats(const uint32_t *list, uint32_t nlist, const uint64_t *lfirst, uint64_t runs,
                            const uint64_t *keys, const uint64_t *ocnt, const uint64_t *leaf_out, uint32_t *leaf_nd,
                            uint64_t *leaf_bytes, uint32_t *leaf_last, unsigned long long *nkeys) {
    const uint32_t k = blockIdx.x;
    const uint64_t lid = list[k];
    const uint64_t D = (k + 1 < nlist ? lfirst[k + 1] : runs) - lfirst[k];
    const uint64_t o0 = leaf_out[lid];
    uint64_t bytes = 0;
    for (uint64_t p = threadIdx.x; p < D; p += blockDim.x)
        bytes += line_len(keys[2 * (o0 + p)], keys[2 * (o0 + p) + 1], ocnt[o0 + p]);
    __shared__ unsigned long long s_b;
    if (threadIdx.x == 0) s_b = 0;
    lds_barrier();
    atomicAdd(&s_b, (unsigned long long)bytes);
    lds_barrier();
    if (threadIdx.x == 0) {
        leaf_nd[lid] = (uint32_t)D;
        leaf_bytes[lid] = s_b;
        leaf_last[lid] = D ? line_len(keys[2 * (o0 + D - 1)], keys[2 * (o0 + D - 1) + 1], ocnt[o0 + D - 1]) : 0u;
        atomicAdd(nkeys, (unsigned long long)D);
    }
}

// weighted keys sorted by (part, key): gather from the aggregated KeySet in sort order
__global__ void k_wweights(const SortRec *r, uint64_t n, KeySet ks, uint64_t *wk0, uint64_t *wk1, uint64_t *wcnt,
                           uint32_t *wpart) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t e = r[i].idx;
    wk0[i] = ks.k0[e];
    wk1[i] = ks.k1[e];
    wcnt[i] = ks.cnt[e];
    wpart[i] = r[i].part;
}

inline dim3 gridw(uint64_t n, int b = 256) { return dim3((unsigned)((n + b - 1) / b)); }

}  // namespace

// ================================================================ host launchers (mrgpu.cpp)
void mrg_wide_launch_counts(const BucketArgs &a, uint64_t *cnt_main, uint64_t *segptr, uint64_t *cnt_flush,
                            hipStream_t s) {
    const uint64_t nsm = 2ull * a.nreg * MRG_NBUCKET + MRG_NBUCKET;
    hipLaunchKernelGGL(k_wmain_counts, gridw(nsm), dim3(256), 0, s, a, cnt_main, segptr);
    hipLaunchKernelGGL(k_wflush_counts, gridw(a.nreg), dim3(256), 0, s, a, cnt_flush);
}
void mrg_wide_launch_flush_gather(const BucketArgs &a, const uint64_t *off, uint64_t *k0, uint64_t *k1, uint32_t *c,
                                  hipStream_t s) {
    hipLaunchKernelGGL(k_wflush_gather, dim3(a.nreg), dim3(256), 0, s, a, off, k0, k1, c);
}
void mrg_wide_launch_sample1(const BucketArgs &a, const uint64_t *off, uint64_t nseg, uint64_t n, uint32_t S,
                             uint32_t R, SortRec *out, hipStream_t s) {
    hipLaunchKernelGGL(k_wsample1, gridw(S), dim3(256), 0, s, a, off, nseg, n, S, R, out);
}
void mrg_wide_launch_split1(const SortRec *smp, uint32_t S, uint32_t R, uint32_t B1r, uint64_t *spl, hipStream_t s) {
    if (B1r > 1) hipLaunchKernelGGL(k_wsplit1, gridw((uint64_t)R * (B1r - 1)), dim3(256), 0, s, smp, S, R, B1r, spl);
}
size_t mrg_wide_l1_lds(uint32_t R, uint32_t B1r, uint32_t B1) {
    return 16ull * R * (B1r - 1u) + 4ull * ((B1 + 1u) & ~1u) + 16ull * W_SEGLDS;
}
void mrg_wide_launch_l1(const BucketArgs &a, const uint64_t *off, const uint64_t *segptr, uint64_t nseg, uint64_t n,
                        const uint64_t *spl1, uint32_t R, uint32_t B1r, uint32_t *cnt, uint32_t ntiles, uint64_t *out,
                        uint16_t *bid, uint8_t *ix1, bool scatter, hipStream_t s) {
    L1Args L{a, off, segptr, nseg, n, spl1, R, B1r, R * B1r, ntiles, cnt, out, bid, nullptr};
    size_t lds = mrg_wide_l1_lds(R, B1r, R * B1r);
    // the counting pass searches the splitters through an index when it fits beside them in LDS
    if (!scatter && ix1 && B1r >= 5 && lds + (size_t)W_IX1 * R <= 160u * 1024u) {
        hipLaunchKernelGGL(k_wl1ix, dim3(R), dim3(320), 0, s, spl1, B1r - 1u, ix1);
        L.ix1 = ix1;
        lds += (size_t)W_IX1 * R;
    }
    if (scatter) hipLaunchKernelGGL(k_wl1<true>, dim3(ntiles), dim3(W_WG), lds, s, L);
    else hipLaunchKernelGGL(k_wl1<false>, dim3(ntiles), dim3(W_WG), lds, s, L);
}
void mrg_wide_launch_bstart(const uint32_t *cnt, uint32_t B1, uint32_t ntiles, uint64_t n, uint64_t *bstart,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_wbstart, gridw(B1 + 1), dim3(256), 0, s, cnt, B1, ntiles, n, bstart);
}
void mrg_wide_launch_l2(const uint64_t *in, uint64_t *out, const uint64_t *bstart, const uint64_t *spl1, uint32_t B1,
                        uint32_t B1r, uint32_t target, uint32_t *nleaf, uint64_t *leaf_lo, uint64_t *leaf_hi,
                        uint64_t *leaf_dlo, uint64_t *leaf_lb, uint16_t *sub, hipStream_t s, const WmapIn &wm,
                        const L2Sparse &sp) {
    L2Args L{in, out, bstart, spl1, B1r, target, nleaf, leaf_lo, leaf_hi, leaf_dlo, leaf_lb, sub,
             wm.rin, wm.soff, wm.grid, wm.wcap, wm.w12, wm.wl16cap, wm.wl16,
             wm.rin && sp.on ? 1u : 0u, sp.capmul, sp.capadd, sp.sample_min, 0u, sp.redo_flags};
    if (wm.rin) {
        hipLaunchKernelGGL(k_wl2<true>, dim3(B1), dim3(W_WG), 0, s, L);
        if (L.sparse) {  // the buckets whose sampled leaves overflowed, with the exact histogram
            L.redo = 1u;
            hipLaunchKernelGGL(k_wl2<true>, dim3(B1), dim3(W_WG), 0, s, L);
        }
    } else {
        hipLaunchKernelGGL(k_wl2<false>, dim3(B1), dim3(W_WG), 0, s, L);
    }
}
// diagnostic builds (-DMRG_WIDE_PROF): the L2 phase clocks summed so far (else zeros)
void mrg_wide_l2_prof(unsigned long long out[8]) {
#ifdef MRG_WIDE_PROF
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_l2prof), 8 * sizeof(unsigned long long));
#else
    for (int i = 0; i < 8; ++i) out[i] = 0;
#endif
}
void mrg_wide_launch_weights(const SortRec *r, uint64_t n, KeySet ks, uint64_t *wk0, uint64_t *wk1, uint64_t *wcnt,
                             uint32_t *wpart, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_wweights, gridw(n), dim3(256), 0, s, r, n, ks, wk0, wk1, wcnt, wpart);
}
void mrg_wide_launch_leaf(const WideLeafArgs &w, uint32_t B1, hipStream_t s) {
    LeafArgs L{w.kin, w.kout, w.bstart, w.nleaf, w.leaf_lo, w.leaf_lb, w.B1r, w.R, w.wk0, w.wk1, w.wcnt, w.wpart, w.nw,
               w.maxd ? min(w.maxd, W_MAXD) : W_MAXD, w.ocnt, w.leaf_out, w.leaf_nd, w.leaf_bytes, w.leaf_last, w.ovf_list,
               w.ovf_n, w.nkeys, w.wr, w.prof, w.big_list, w.big_n, w.leaf_pk, w.pack, w.leaf_hi, w.leaf_dlo};
    hipLaunchKernelGGL(k_wranges, gridw((uint64_t)B1 * MRG_WIDE_MAXB2), dim3(256), 0, s, L, B1);
    hipLaunchKernelGGL(k_wleafw, dim3(B1 * W_VQ), dim3(64), 0, s, L);
    // the passed-on leaves: a fixed grid loops over the list (its length is read on the device)
    hipLaunchKernelGGL(k_wleaf, dim3(B1 < 2048u ? B1 : 2048u), dim3(W_LWG), 0, s, L);
}
void mrg_wide_launch_fallback(const WideLeafArgs &w, const uint32_t *list, uint32_t nlist, DevPool &pool,
                              hipStream_t s) {
    LeafArgs L{w.kin, w.kout, w.bstart, w.nleaf, w.leaf_lo, w.leaf_lb, w.B1r, w.R, w.wk0, w.wk1, w.wcnt, w.wpart, w.nw,
               w.maxd ? min(w.maxd, W_MAXD) : W_MAXD, w.ocnt, w.leaf_out, w.leaf_nd, w.leaf_bytes, w.leaf_last, w.ovf_list,
               w.ovf_n, w.nkeys, w.wr, w.prof, w.big_list, w.big_n, w.leaf_pk, w.pack, w.leaf_hi, w.leaf_dlo};
    uint64_t *wrange = (uint64_t *)pool.get(16ull * nlist);
    uint64_t *cnt = (uint64_t *)pool.get(8ull * (nlist + 1)), *off = (uint64_t *)pool.get(8ull * (nlist + 1));
    uint64_t *scantmp = (uint64_t *)pool.get(8ull * mrg_scan_tmp_elems(nlist + 1));
    hipLaunchKernelGGL(k_wfb_wrange, gridw(nlist), dim3(256), 0, s, L, list, nlist, wrange);
    hipMemsetAsync(cnt + nlist, 0, 8, s);
    hipLaunchKernelGGL(k_wfb_count, gridw(nlist), dim3(256), 0, s, list, nlist, w.leaf_lo, w.leaf_hi, wrange, cnt);
    mrg_scan_u64(cnt, off, nlist + 1, scantmp, s);
    uint64_t n = 0;
    hipMemcpyAsync(&n, off + nlist, 8, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    SortRec *a = (SortRec *)pool.get(sizeof(SortRec) * (n + 1)), *b = (SortRec *)pool.get(sizeof(SortRec) * (n + 1));
    uint64_t *rcnt = (uint64_t *)pool.get(8ull * (n + 1));
    hipLaunchKernelGGL(k_wfb_gather, dim3(nlist), dim3(256), 0, s, list, off, w.leaf_lo, w.leaf_hi, wrange,
                       w.kin, w.wk0, w.wk1, w.wcnt, a, rcnt);
    SortPlan plan{};
    plan.use_part = nlist > 1;
    uint32_t pb = 0;
    for (uint32_t v = nlist - 1; v; v >>= 8) ++pb;
    plan.part_bytes = pb;
    plan.use_k0 = plan.use_k1 = true;
    void *stmp = pool.get(mrg_sort_tmp_bytes(n));
    int passes = 0;
    SortRec *srt = mrg_radix_sort(a, b, n, plan, stmp, s, &passes);
    uint64_t *head = (uint64_t *)pool.get(8ull * (n + 1)), *E = (uint64_t *)pool.get(8ull * (n + 1));
    uint64_t *lfirst = (uint64_t *)pool.get(8ull * (nlist + 1));
    uint64_t *scantmp2 = (uint64_t *)pool.get(8ull * mrg_scan_tmp_elems(n + 1));
    hipLaunchKernelGGL(k_wfb_heads, gridw(n), dim3(256), 0, s, srt, n, head);
    mrg_scan_u64(head, E, n, scantmp2, s);
    hipLaunchKernelGGL(k_wfb_lfirst, gridw(n), dim3(256), 0, s, srt, n, head, E, lfirst);
    uint64_t tail[2] = {0, 0};
    hipMemcpyAsync(&tail[0], E + (n - 1), 8, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(&tail[1], head + (n - 1), 8, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    const uint64_t runs = tail[0] + tail[1];
    hipLaunchKernelGGL(k_wfb_emit, gridw(n), dim3(256), 0, s, srt, n, head, E, rcnt, list, lfirst, w.leaf_out, w.kout,
                       w.ocnt);
    hipLaunchKernelGGL(k_wfb_stats, dim3(nlist), dim3(256), 0, s, list, nlist, lfirst, runs, w.kout, w.ocnt, w.leaf_out,
                       w.leaf_nd, w.leaf_bytes, w.leaf_last, w.nkeys);
    hipStreamSynchronize(s);
    pool.put(wrange); pool.put(cnt); pool.put(off); pool.put(scantmp); pool.put(a); pool.put(b); pool.put(rcnt);
    pool.put(stmp); pool.put(head); pool.put(E); pool.put(lfirst); pool.put(scantmp2);
}
void mrg_wide_launch_drop(const uint32_t *nleaf, uint32_t B1r, uint32_t R, const uint32_t *leaf_nd, uint64_t *leaf_bytes,
                          const uint32_t *leaf_last, uint32_t *leaf_drop, hipStream_t s) {
    hipLaunchKernelGGL(k_wdrop, gridw(R), dim3(256), 0, s, nleaf, B1r, R, leaf_nd, leaf_bytes, leaf_last, leaf_drop);
}
void mrg_wide_launch_write(const uint64_t *keys, const uint64_t *ocnt, const uint32_t *leaf_pk, const uint32_t *nleaf,
                           const uint64_t *leaf_out, const uint32_t *leaf_nd, const uint32_t *leaf_drop,
                           const uint64_t *leaf_off, uint32_t B1, uint8_t *out, hipStream_t s) {
#if MRG_WIDE_WWAVE
    hipLaunchKernelGGL(k_wwritew, dim3(B1 * WW_PER), dim3(WW_WG), 0, s, keys, ocnt, leaf_pk, nleaf, leaf_out, leaf_nd,
                       leaf_drop, leaf_off, out);
#else
    hipLaunchKernelGGL(k_wwrite, dim3(B1), dim3(W_WWG), 0, s, keys, ocnt, leaf_pk, nleaf, leaf_out, leaf_nd, leaf_drop,
                       leaf_off, out);
#endif
}
void mrg_wide_launch_part_off(const uint64_t *leaf_off, uint32_t B1r, uint32_t R, uint64_t total, uint64_t *part_off,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_wpart_off, gridw(R + 1), dim3(256), 0, s, leaf_off, B1r, R, total, part_off);
}
void mrg_wide_launch_dense(const uint64_t *keys, const uint64_t *ocnt, const uint32_t *leaf_pk, const uint64_t *leaf_out,
                           const uint32_t *leaf_nd, const uint32_t *dense_off, uint32_t B1, uint32_t B1r, KeySet ks,
                           hipStream_t s) {
    hipLaunchKernelGGL(k_wdense, dim3(B1 * MRG_WIDE_MAXB2), dim3(256), 0, s, keys, ocnt, leaf_pk, leaf_out, leaf_nd,
                       dense_off, B1r, ks);
}

void mrg_wide_launch_sample_text(const uint8_t *in, const uint64_t *doc_off, uint32_t n_docs, uint64_t total,
                                 uint32_t S, uint32_t R, SortRec *out, hipStream_t s) {
    if (S) hipLaunchKernelGGL(k_wsample_text, dim3((S + 255) / 256), dim3(256), 0, s, in, doc_off, n_docs, total, S, R,
                              out);
}
void mrg_wide_launch_sample_uniq(const SortRec *r, uint32_t S, unsigned long long *dups, hipStream_t s) {
    if (S > W_UQ / 2) S = W_UQ / 2;
    hipLaunchKernelGGL(k_wsample_uniq, dim3(1), dim3(1024), 0, s, r, S, dups);
}
void mrg_wide_launch_sample_dups(const SortRec *r, uint32_t S, unsigned long long *dups, hipStream_t s) {
    if (S) hipLaunchKernelGGL(k_wsample_dups, dim3((S + 255) / 256), dim3(256), 0, s, r, S, dups);
}
void mrg_wide_launch_l1ix(const uint64_t *spl1, uint32_t R, uint32_t B1r, uint8_t *ix1, hipStream_t s) {
    if (B1r > 1) hipLaunchKernelGGL(k_wl1ix, dim3(R), dim3(256), 0, s, spl1, B1r - 1u, ix1);
}
void mrg_wmap_launch_seg(const uint32_t *wcnt, uint32_t B1, uint32_t grid, uint32_t wcap, const uint32_t *wl16n,
                         uint32_t wl16cap, uint32_t *soff, uint64_t *nb, hipStream_t s) {
    hipLaunchKernelGGL(k_wmap_seg, dim3(B1), dim3(64), 0, s, wcnt, grid, wcap, wl16n, wl16cap, soff, nb);
}
