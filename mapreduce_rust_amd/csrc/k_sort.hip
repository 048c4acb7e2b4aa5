// k_sort.hip -- device-wide exclusive scan and stable LSD radix sort (8-bit digits) for gfx950.
//
// Replaces the reduce-side key_value_contents.sort_by(|a, b| a.key.cmp(&b.key)) (src/mr/worker.rs:
// 162-164) for the DISTINCT keys of the owned partitions, and sorts long-key fingerprints for the
// collision-safe grouping.  One upfront kernel builds the digit histograms of every pass; passes
// whose digit is constant are skipped (e.g. key bytes beyond the longest key, nReduce <= 256).
// Per pass: per-tile histogram -> scan -> stable scatter, the local rank computed by a wave64
// 8-ballot match (peers with the same digit) plus per-wave digit counters in LDS.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "mrg_device.h"
#include "mrg_internal.h"

namespace {

constexpr int BS = 256;                 // threads per block
constexpr int IPT = 8;                  // items per thread
constexpr int TILE = BS * IPT;          // 2048 items per tile

// ------------------------------------------------------------------ block scan helpers
template <class T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const int lane = __lane_id();
    for (int o = 1; o < 64; o <<= 1) {
        const T u = __shfl_up(v, o);
        if (lane >= o) v += u;
    }
    return v;
}

// exclusive scan across the block of one value per thread; returns exclusive prefix, *total = sum
template <class T>
__device__ __forceinline__ T block_excl_scan(T v, T *s_wave, T *total) {
    const int lane = __lane_id(), w = threadIdx.x >> 6;
    const T inc = wave_incl_scan(v);
    if (lane == 63) s_wave[w] = inc;
    __syncthreads();
    T base = 0, tot = 0;
    for (int i = 0; i < BS / 64; ++i) {
        const T x = s_wave[i];
        if (i < w) base += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return base + inc - v;
}

template <class T>
__global__ void k_scan_tile_sums(const T *in, uint64_t n, T *sums) {
    __shared__ T s_wave[BS / 64];
    const uint64_t base = (uint64_t)blockIdx.x * TILE + (uint64_t)threadIdx.x * IPT;
    T v = 0;
    for (int k = 0; k < IPT; ++k)
        if (base + k < n) v += in[base + k];
    T tot;
    block_excl_scan(v, s_wave, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// exclusive scan of each tile, plus tile prefix (from `prefix`, may be null)
template <class T>
__global__ void k_scan_tiles(const T *in, T *out, uint64_t n, const T *prefix) {
    __shared__ T s_wave[BS / 64];
    const uint64_t base = (uint64_t)blockIdx.x * TILE + (uint64_t)threadIdx.x * IPT;
    T x[IPT];
    T v = 0;
    for (int k = 0; k < IPT; ++k) {
        x[k] = base + k < n ? in[base + k] : (T)0;
        v += x[k];
    }
    T tot;
    T run = block_excl_scan(v, s_wave, &tot);
    if (prefix) run += prefix[blockIdx.x];
    for (int k = 0; k < IPT; ++k) {
        if (base + k < n) out[base + k] = run;
        run += x[k];
    }
}

template <class T>
void scan_rec(const T *in, T *out, uint64_t n, T *tmp, hipStream_t s) {
    if (!n) return;
    const uint64_t nt = (n + TILE - 1) / TILE;
    if (nt == 1) {
        hipLaunchKernelGGL(k_scan_tiles<T>, dim3(1), dim3(BS), 0, s, in, out, n, (const T *)nullptr);
        return;
    }
    T *sums = tmp;
    T *rest = tmp + nt;
    hipLaunchKernelGGL(k_scan_tile_sums<T>, dim3((unsigned)nt), dim3(BS), 0, s, in, n, sums);
    scan_rec<T>(sums, sums, nt, rest, s);
    hipLaunchKernelGGL(k_scan_tiles<T>, dim3((unsigned)nt), dim3(BS), 0, s, in, out, n, (const T *)sums);
}

uint64_t scan_tmp(uint64_t n) {
    uint64_t t = 0;
    while (n > TILE) {
        n = (n + TILE - 1) / TILE;
        t += n;
    }
    return t + 16;
}

// ------------------------------------------------------------------ radix sort
struct RecTraits {  // SortRec, key = (part, k0, k1, doc); pass q counts bytes from the LSB end
    using R = SortRec;
    static constexpr int NPASS = 24;
    __device__ static __forceinline__ uint32_t digit(const R &r, int q) {
        if (q < 4) return (r.doc >> (8 * q)) & 0xFFu;
        if (q < 12) return (uint32_t)(r.k1 >> (8 * (q - 4))) & 0xFFu;
        if (q < 20) return (uint32_t)(r.k0 >> (8 * (q - 12))) & 0xFFu;
        return (r.part >> (8 * (q - 20))) & 0xFFu;
    }
};
struct KV64 {
    uint64_t key;
    uint32_t val, pad;
};
struct KVTraits {
    using R = KV64;
    static constexpr int NPASS = 8;
    __device__ static __forceinline__ uint32_t digit(const R &r, int q) { return (uint32_t)(r.key >> (8 * q)) & 0xFFu; }
};

// all-pass histograms in one read: hist[q * 256 + d], for the passes in qmask only.  A digit that
// is the same on every active lane (constant bytes: zero padding of short keys, the partition's
// high bytes) is added once by the first lane instead of by 64 lanes on one LDS address.
template <class TR>
__global__ void k_all_hist(const typename TR::R *in, uint64_t n, unsigned long long *hist, uint32_t qmask) {
    __shared__ unsigned int s_h[TR::NPASS * 256];
    for (int i = threadIdx.x; i < TR::NPASS * 256; i += BS) s_h[i] = 0;
    __syncthreads();
    const uint32_t lane = __lane_id();
    for (uint64_t i = (uint64_t)blockIdx.x * BS + threadIdx.x; i < n; i += (uint64_t)gridDim.x * BS) {
        const typename TR::R r = in[i];
        const uint64_t act = __ballot(1);
        const uint32_t first = (uint32_t)__ffsll((unsigned long long)act) - 1u;
        for (int q = 0; q < TR::NPASS; ++q) {
            if (!((qmask >> q) & 1u)) continue;
            const uint32_t d = TR::digit(r, q);
            const uint32_t d0 = __builtin_amdgcn_readfirstlane(d);
            if (__ballot(d == d0) == act) {
                if (lane == first) atomicAdd(&s_h[q * 256 + d0], (unsigned int)__popcll(act));
            } else {
                atomicAdd(&s_h[q * 256 + d], 1u);
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < TR::NPASS * 256; i += BS)
        if (s_h[i]) atomicAdd(&hist[i], (unsigned long long)s_h[i]);
}

// per-tile digit counts, digit-major: cnt[d * ntiles + tile]
template <class TR>
__global__ void k_tile_hist(const typename TR::R *in, uint64_t n, int q, uint32_t *cnt, uint32_t ntiles) {
    __shared__ unsigned int s_h[256];
    s_h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    for (int k = 0; k < IPT; ++k) {
        const uint64_t i = base + (uint64_t)k * BS + threadIdx.x;
        if (i < n) atomicAdd(&s_h[TR::digit(in[i], q)], 1u);
    }
    __syncthreads();
    cnt[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = s_h[threadIdx.x];
}

// stable scatter: item order inside a tile is (round k, thread t) = base + k*BS + t, exactly the
// order the ranks are assigned in
template <class TR>
__global__ void k_scatter(const typename TR::R *in, typename TR::R *out, uint64_t n, int q, const uint32_t *off,
                          uint32_t ntiles) {
    __shared__ uint32_t s_base[256];
    __shared__ uint32_t s_run[256];
    __shared__ uint32_t s_wc[BS / 64][256];
    const int t = threadIdx.x, w = t >> 6;
    s_base[t] = off[(uint64_t)t * ntiles + blockIdx.x];
    s_run[t] = 0;
    for (int i = 0; i < BS / 64; ++i) s_wc[i][t] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * TILE;
    const uint64_t lt = mrg_lanemask_lt();
    for (int k = 0; k < IPT; ++k) {
        const uint64_t i = base + (uint64_t)k * BS + t;
        const bool valid = i < n;
        typename TR::R r;
        uint32_t d = 0;
        if (valid) {
            r = in[i];
            d = TR::digit(r, q);
        }
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < 8; ++b) {
            const uint64_t m = __ballot(valid && ((d >> b) & 1u));
            peers &= ((d >> b) & 1u) ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        if (valid && rank == 0) s_wc[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = s_base[d] + s_run[d] + rank;
            for (int i2 = 0; i2 < w; ++i2) pos += s_wc[i2][d];
            out[pos] = r;
        }
        __syncthreads();
        {
            uint32_t add = 0;
            for (int i2 = 0; i2 < BS / 64; ++i2) {
                add += s_wc[i2][t];
                s_wc[i2][t] = 0;
            }
            s_run[t] += add;
        }
        __syncthreads();
    }
}

template <class TR>
typename TR::R *radix_sort_t(typename TR::R *a, typename TR::R *b, uint64_t n, const bool *want, void *tmp,
                             hipStream_t s, int *passes_run) {
    if (passes_run) *passes_run = 0;
    if (n <= 1) return a;
    const uint32_t ntiles = (uint32_t)((n + TILE - 1) / TILE);
    unsigned long long *hist = (unsigned long long *)tmp;
    uint32_t *cnt = (uint32_t *)(hist + TR::NPASS * 256);
    uint32_t *scantmp = cnt + (uint64_t)256 * ntiles;
    hipMemsetAsync(hist, 0, sizeof(unsigned long long) * TR::NPASS * 256, s);
    const unsigned g = (unsigned)std::min<uint64_t>((n + BS - 1) / BS, 1024);
    uint32_t qmask = 0;
    for (int q = 0; q < TR::NPASS; ++q)
        if (want[q]) qmask |= 1u << q;
    hipLaunchKernelGGL(k_all_hist<TR>, dim3(g), dim3(BS), 0, s, a, n, hist, qmask);
    unsigned long long h[TR::NPASS * 256];
    hipMemcpyAsync(h, hist, sizeof h, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    for (int q = 0; q < TR::NPASS; ++q) {
        if (!want[q]) continue;
        bool trivial = false;
        for (int d = 0; d < 256; ++d)
            if (h[q * 256 + d] == n) { trivial = true; break; }
        if (trivial) continue;
        hipLaunchKernelGGL(k_tile_hist<TR>, dim3(ntiles), dim3(BS), 0, s, a, n, q, cnt, ntiles);
        scan_rec<uint32_t>(cnt, cnt, (uint64_t)256 * ntiles, scantmp, s);
        hipLaunchKernelGGL(k_scatter<TR>, dim3(ntiles), dim3(BS), 0, s, a, b, n, q, cnt, ntiles);
        std::swap(a, b);
        if (passes_run) ++*passes_run;
    }
    return a;
}

// ------------------------------------------------------------------ MSD bucket sort of SortRecs
// The distinct keys of a job (~1e6) sorted by (part, k0, k1, doc) in three passes instead of up to
// 13 LSD passes: every record takes a bucket = (part, leading key bits) and its rank inside the
// bucket from one global atomic; the buckets' offsets are scanned; records are scattered; then each
// bucket is sorted on its own: buckets of at most 64 records by ONE WAVE (rank by comparison with
// every record of the bucket, broadcast from its lane: no LDS, no barrier -- with 2^20 bucket ids
// most buckets of text keys are this small), larger ones of at most MSD_LCAP records by one
// workgroup (bitonic network over whole records in LDS).  The key bits of the bucket id come from
// the first three key bytes clamped to 7 bits (monotone: every byte >= 0x7F maps to 0x7F), so text
// keys, whose bytes leave the top bit unused, spread over the buckets.  A few oversized buckets are
// sorted by the LSD radix sort on their own segments; many of them (a skewed key set) send the whole
// array through the LSD sort.  Records compare by (part, k0, k1, doc, idx): idx is unique, so the
// order is total even for > 16-byte keys with equal prefixes (k_fix_runs orders those afterwards).
constexpr int MSD_BITS = 20;
constexpr uint32_t MSD_NB = 1u << MSD_BITS;
constexpr int MSD_WG = 256;
constexpr uint32_t MSD_GRID = 1024;  // leaf workgroups (they stride over the bucket lists)
constexpr uint32_t MSD_LCAP = 2048;
constexpr uint32_t MSD_SMALL = 64;   // buckets sorted by one wave
constexpr uint32_t MSD_SMALL_GRID = 2048;  // workgroups of the one-wave leaf kernel
constexpr uint32_t MSD_MAX_BIG = 16;

__device__ __forceinline__ uint32_t msd_bucket(const SortRec &r, uint32_t pbits) {
    if (pbits >= (uint32_t)MSD_BITS) return r.part >> (pbits - MSD_BITS);
    // bytes clamped to 7 bits, saturating: after a byte >= 0x7F every later byte counts as 0x7F
    // (otherwise "\xc3\x86n" would get a larger code than "\xc3\x88")
    const uint32_t c0 = (uint32_t)(r.k0 >> 56), c1 = (uint32_t)(r.k0 >> 48) & 0xFFu, c2 = (uint32_t)(r.k0 >> 40) & 0xFFu;
    const uint32_t b0 = min(c0, 127u);
    const uint32_t b1 = b0 == 127u ? 127u : min(c1, 127u);
    const uint32_t b2 = b1 == 127u ? 127u : min(c2, 127u);
    const uint32_t code = (b0 << 14) | (b1 << 7) | b2;  // 21 bits, monotone in the key
    const uint32_t kb = MSD_BITS - pbits;              // key bits of the bucket id (1..20)
    return (r.part << kb) | (code >> (21 - kb));
}

__device__ __forceinline__ uint32_t uni_lane(uint32_t v, uint32_t j) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)j);
}

__device__ __forceinline__ bool rec_less(const SortRec &a, const SortRec &b) {
    if (a.part != b.part) return a.part < b.part;
    if (a.k0 != b.k0) return a.k0 < b.k0;
    if (a.k1 != b.k1) return a.k1 < b.k1;
    if (a.doc != b.doc) return a.doc < b.doc;
    return a.idx < b.idx;
}

__global__ void k_msd_count(const SortRec *in, uint64_t n, uint32_t pbits, uint32_t *cnt, uint32_t *rank,
                            uint32_t *zero0, uint32_t *zero1, uint32_t *zero2) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) {  // the later kernels' counters (list lengths, oversized count): no memset launches
        *zero0 = 0;
        *zero1 = 0;
        *zero2 = 0;
    }
    if (i >= n) return;
    rank[i] = atomicAdd(&cnt[msd_bucket(in[i], pbits)], 1u);
}

__global__ void k_msd_scatter(const SortRec *in, SortRec *out, uint64_t n, uint32_t pbits, const uint32_t *off,
                              const uint32_t *rank) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SortRec r = in[i];
    out[off[msd_bucket(r, pbits)] + rank[i]] = r;
}

// The buckets with at least 2 records, listed (list[0] = how many): at most `small` records in
// list (one wave each), more in list2 (one workgroup each).  The leaf kernels share the work by list
// position, not by bucket id (bucket ids of text keys cluster in a few ranges).
__global__ __launch_bounds__(1024) void k_msd_list(const uint32_t *off, uint32_t small, uint32_t *list, uint32_t *list2) {
    // 1024 buckets per workgroup: ranks inside the workgroup through LDS, one device atomic per list
    __shared__ uint32_t s_n[2], s_base[2];
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t m = b < MSD_NB ? off[b + 1] - off[b] : 0u;
    const uint32_t lane = __lane_id();
    if (threadIdx.x < 2) s_n[threadIdx.x] = 0;
    __syncthreads();
    const bool p1 = m >= 2u && m <= small, p2 = m > small;
    uint32_t r1 = 0, r2 = 0;
    auto rank = [&](bool pred, uint32_t k) -> uint32_t {
        const uint64_t msk = __ballot(pred);
        if (!msk) return 0;
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)msk) - 1u;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&s_n[k], (uint32_t)__popcll(msk));
        base = __shfl(base, (int)leader);
        return base + (uint32_t)__popcll(msk & mrg_lanemask_lt());
    };
    r1 = rank(p1, 0);
    r2 = rank(p2, 1);
    __syncthreads();
    if (threadIdx.x == 0 && s_n[0]) s_base[0] = atomicAdd(&list[0], s_n[0]);
    if (threadIdx.x == 64 && s_n[1]) s_base[1] = atomicAdd(&list2[0], s_n[1]);
    __syncthreads();
    if (p1) list[1 + s_base[0] + r1] = b;
    if (p2) list2[1 + s_base[1] + r2] = b;
}

// One wave per small bucket (m <= 64): lane i holds record i; its rank = the records of the bucket
// that order before it (each broadcast from its lane in turn; idx makes the order total), then every
// record is stored at its rank.
__global__ __launch_bounds__(MSD_WG) void k_msd_leaf_small(SortRec *recs, const uint32_t *off, const uint32_t *list) {
    const uint32_t nl = list[0];
    const uint32_t lane = __lane_id();
    const uint32_t nw = gridDim.x * (MSD_WG / 64);
    auto uni = [](uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
    for (uint32_t x = uni(blockIdx.x * (MSD_WG / 64) + (threadIdx.x >> 6)); x < nl; x += nw) {
        const uint32_t b = uni(list[1 + x]);
        const uint32_t lo = uni(off[b]), m = uni(off[b + 1]) - lo;
        SortRec r{};
        if (lane < m) r = recs[lo + lane];
        uint32_t rank = 0;
        for (uint32_t j = 0; j < m; ++j) {  // wave-uniform trip count; branch-free compare
            const uint64_t k0 = ((uint64_t)uni_lane((uint32_t)(r.k0 >> 32), j) << 32) | uni_lane((uint32_t)r.k0, j);
            const uint64_t k1 = ((uint64_t)uni_lane((uint32_t)(r.k1 >> 32), j) << 32) | uni_lane((uint32_t)r.k1, j);
            const uint32_t pt = uni_lane(r.part, j), dc = uni_lane(r.doc, j), ix = uni_lane(r.idx, j);
            const bool lt = (pt < r.part) |
                            ((pt == r.part) & ((k0 < r.k0) | ((k0 == r.k0) & ((k1 < r.k1) | ((k1 == r.k1) &
                            ((dc < r.doc) | ((dc == r.doc) & (ix < r.idx))))))));
            rank += lt ? 1u : 0u;
        }
        if (lane < m) recs[lo + rank] = r;
    }
}

// workgroups stride over the large-bucket list: each bucket's records through LDS, bitonic-sorted
// (padding sorts last); an oversized bucket is only listed (big[0] = how many, big[1..] = which, up
// to MSD_MAX_BIG)
__global__ __launch_bounds__(MSD_WG) void k_msd_leaf(SortRec *recs, const uint32_t *off, const uint32_t *list,
                                                    uint32_t lcap, uint32_t *big) {
    __shared__ SortRec s_r[MSD_LCAP];
    const uint32_t nl = list[0];
    for (uint32_t x = blockIdx.x; x < nl; x += gridDim.x) {
        const uint32_t b = list[1 + x];
        const uint32_t lo = off[b], m = off[b + 1] - lo;
        if (m > lcap) {
            if (threadIdx.x == 0) {
                const uint32_t k = atomicAdd(&big[0], 1u);
                if (k < MSD_MAX_BIG) big[1 + k] = b;
            }
            continue;
        }
        uint32_t P = 2;
        while (P < m) P <<= 1;
        for (uint32_t i = threadIdx.x; i < P; i += MSD_WG) {
            SortRec r;
            if (i < m) r = recs[lo + i];
            else r = SortRec{~0ull, ~0ull, ~0u, ~0u, ~0u, 0u};
            s_r[i] = r;
        }
        __syncthreads();
        for (uint32_t k = 2; k <= P; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                for (uint32_t t = threadIdx.x; t < P / 2; t += MSD_WG) {
                    const uint32_t i = 2 * t - (t & (j - 1)), l = i + j;
                    const SortRec x = s_r[i], y = s_r[l];
                    if (rec_less(y, x) == ((i & k) == 0)) {
                        s_r[i] = y;
                        s_r[l] = x;
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t i = threadIdx.x; i < m; i += MSD_WG) recs[lo + i] = s_r[i];
        __syncthreads();  // s_r is reused by the next bucket
    }
}

__global__ void k_pack_kv(const uint64_t *k, const uint32_t *v, uint64_t n, KV64 *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = KV64{k[i], v[i], 0};
}
__global__ void k_unpack_kv(const KV64 *in, uint64_t n, uint64_t *k, uint32_t *v) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { k[i] = in[i].key; v[i] = in[i].val; }
}

}  // namespace

uint64_t mrg_scan_tmp_elems(uint64_t n) { return scan_tmp(n); }

void mrg_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *tmp, hipStream_t s) {
    scan_rec<uint64_t>(in, out, n, tmp, s);
}

void mrg_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *tmp, hipStream_t s) {
    scan_rec<uint32_t>(in, out, n, tmp, s);
}

uint64_t mrg_sort_tmp_bytes(uint64_t n) {
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    const uint64_t lsd = sizeof(unsigned long long) * 24 * 256 + sizeof(uint32_t) * (256 * ntiles + scan_tmp(256 * ntiles)) + 256;
    const uint64_t msd = sizeof(uint32_t) * (4ull * (MSD_NB + 2) + MSD_MAX_BIG + 2 + scan_tmp(MSD_NB + 1) + n) + 256;
    return lsd + msd + 256;  // the MSD arrays, then room for an LSD sort of one oversized bucket
}

struct MsdTmp {
    uint32_t *cnt, *off, *big, *list, *list2, *stmp, *rank;
    void *ltmp;
};
static MsdTmp msd_tmp(void *tmp, uint64_t n) {
    MsdTmp t;
    t.cnt = (uint32_t *)tmp;                 // [NB + 1]
    t.off = t.cnt + (MSD_NB + 2);            // [NB + 1]
    t.big = t.off + (MSD_NB + 2);            // [1 + MAX_BIG]
    t.list = t.big + (MSD_MAX_BIG + 2);      // [1 + NB] buckets of 2..small records
    t.list2 = t.list + (MSD_NB + 2);         // [1 + NB] larger buckets
    t.stmp = t.list2 + (MSD_NB + 2);         // scan temp
    t.rank = t.stmp + scan_tmp(MSD_NB + 1);
    // the LSD temp (histograms, tile counts) goes after the MSD arrays
    t.ltmp = (void *)(((uintptr_t)(t.rank + n) + 255) & ~(uintptr_t)255);
    return t;
}

void mrg_msd_sort_launch(SortRec *a, SortRec *b, uint64_t n, uint32_t pbits, void *tmp, hipStream_t s,
                         uint32_t *h_nbig) {
    *h_nbig = 0;
    if (n <= 1) return;
    const MsdTmp t = msd_tmp(tmp, n);
    hipMemsetAsync(t.cnt, 0, sizeof(uint32_t) * (MSD_NB + 2), s);
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_msd_count, dim3(g), dim3(256), 0, s, a, n, pbits, t.cnt, t.rank, t.big, t.list, t.list2);
    scan_rec<uint32_t>(t.cnt, t.off, MSD_NB + 1, t.stmp, s);  // off[NB] = n (cnt[NB] == 0)
    hipLaunchKernelGGL(k_msd_scatter, dim3(g), dim3(256), 0, s, a, b, n, pbits, t.off, t.rank);
    uint32_t lcap = MSD_LCAP;
    if (const char *e = getenv("MRG_TEST_SORT_LCAP")) lcap = std::max<uint32_t>(1u, std::min<uint32_t>(MSD_LCAP, (uint32_t)atoi(e)));
    hipLaunchKernelGGL(k_msd_list, dim3(MSD_NB / 1024), dim3(1024), 0, s, t.off, std::min(MSD_SMALL, lcap), t.list, t.list2);
    // small buckets: one wave each, 8 workgroups (32 waves) per CU striding over the list (the
    // list length is on the device; a grid of n / 2 waves spent its time dispatching empty waves)
    const uint64_t nsmall = std::min<uint64_t>(n / 2, (uint64_t)MSD_SMALL_GRID * (MSD_WG / 64));
    hipLaunchKernelGGL(k_msd_leaf_small, dim3((unsigned)((nsmall + MSD_WG / 64 - 1) / (MSD_WG / 64))), dim3(MSD_WG), 0, s,
                       b, t.off, t.list);
    hipLaunchKernelGGL(k_msd_leaf, dim3(MSD_GRID), dim3(MSD_WG), 0, s, b, t.off, t.list2, lcap, t.big);
    hipMemcpyAsync(h_nbig, t.big, sizeof(uint32_t), hipMemcpyDeviceToHost, s);  // pinned: no wait here
}

SortRec *mrg_msd_sort_finish(SortRec *a, SortRec *b, uint64_t n, const SortPlan &plan, void *tmp, hipStream_t s,
                             uint32_t nb) {
    if (n <= 1) return a;
    if (!nb) return b;
    const MsdTmp t = msd_tmp(tmp, n);
    if (nb > MSD_MAX_BIG) return mrg_radix_sort(b, a, n, plan, t.ltmp, s, nullptr);  // skewed: all of it
    std::vector<uint32_t> bl(nb), o(MSD_NB + 1);
    hipMemcpyAsync(bl.data(), t.big + 1, sizeof(uint32_t) * nb, hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(o.data(), t.off, sizeof(uint32_t) * (MSD_NB + 1), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    for (uint32_t bk : bl) {  // each oversized bucket by the LSD sort on its segment (a: scratch)
        const uint64_t lo = o[bk], m = o[bk + 1] - lo;
        SortRec *r = mrg_radix_sort(b + lo, a + lo, m, plan, t.ltmp, s, nullptr);
        if (r != b + lo) hipMemcpyAsync(b + lo, r, sizeof(SortRec) * m, hipMemcpyDeviceToDevice, s);
    }
    return b;
}

SortRec *mrg_msd_sort(SortRec *a, SortRec *b, uint64_t n, uint32_t pbits, const SortPlan &plan, void *tmp,
                      hipStream_t s, uint32_t *n_big, uint32_t *h_pinned) {
    mrg_msd_sort_launch(a, b, n, pbits, tmp, s, h_pinned);
    hipStreamSynchronize(s);
    const uint32_t nb = *h_pinned;
    if (n_big) *n_big = nb;
    return mrg_msd_sort_finish(a, b, n, plan, tmp, s, nb);
}

SortRec *mrg_radix_sort(SortRec *recs, SortRec *alt, uint64_t n, const SortPlan &plan, void *tmp, hipStream_t s,
                        int *passes_run) {
    bool want[24];
    for (int q = 0; q < 24; ++q) {
        if (q < 4) want[q] = plan.use_doc && (uint32_t)q < plan.doc_bytes;
        else if (q < 12) want[q] = plan.use_k1;
        else if (q < 20) want[q] = plan.use_k0;
        else want[q] = plan.use_part && (uint32_t)(q - 20) < plan.part_bytes;
    }
    return radix_sort_t<RecTraits>(recs, alt, n, want, tmp, s, passes_run);
}

// (key, val) pairs sorted by key, stable, in place; kv_tmp holds two KV64 staging arrays (4n u64).
void mrg_radix_sort_u64(uint64_t *keys, uint32_t *vals, uint64_t *kv_tmp, uint64_t n, void *tmp, hipStream_t s) {
    if (n <= 1) return;
    KV64 *a = (KV64 *)kv_tmp;
    KV64 *b = a + n;
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_pack_kv, dim3(g), dim3(256), 0, s, keys, vals, n, a);
    bool want[8];
    for (int q = 0; q < 8; ++q) want[q] = true;
    KV64 *r = radix_sort_t<KVTraits>(a, b, n, want, tmp, s, nullptr);
    hipLaunchKernelGGL(k_unpack_kv, dim3(g), dim3(256), 0, s, r, n, keys, vals);
}
