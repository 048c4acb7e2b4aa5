// k_keys.hip -- global aggregation of map records, long-key tie-break grouping, partitioning and
// the shuffle pack (gfx950).
//
// Global table: the reduce side's "group equal keys" (src/mr/worker.rs:165-184) done by hashing
// instead of sorting every record: records from all map workgroups are summed per exact key in an
// HBM open-addressing table with the same monotone claim protocol as the LDS table (k_map.hip):
// device-scope 64-bit CAS per key word, so the table is exact without locks.  Every distinct key
// then gets its partition SipHash-1-3(key ++ 0xFF) % nReduce (worker.rs:111-115, 129) -- once per
// key, not per token.
#include <algorithm>
#include <type_traits>

#include "mrg_device.h"
#include "mrg_internal.h"

namespace {

inline dim3 grid_for(uint64_t n, int b = 256) { return dim3((unsigned)((n + b - 1) / b)); }

// Slot of this thread's item in an append to *counter by the whole workgroup (every thread calls it):
// one device atomic per workgroup instead of one per wave (a table of 2 M slots compacted with a wave
// atomic each spent 0.4 ms on one contended counter).
template <int WG>
__device__ __forceinline__ uint64_t wg_append(unsigned long long *counter, bool pred, uint32_t *s_w,
                                              unsigned long long *s_base) {
    const uint64_t m = __ballot(pred);
    const uint32_t wv = threadIdx.x >> 6, lane = __lane_id();
    if (lane == 0) s_w[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int w = 0; w < WG / 64; ++w) {
            const uint32_t c = s_w[w];
            s_w[w] = run;
            run += c;
        }
        *s_base = run ? atomicAdd(counter, (unsigned long long)run) : 0ull;
    }
    __syncthreads();
    return *s_base + s_w[wv] + (uint64_t)__popcll(m & mrg_lanemask_lt());
}

// ---------------------------------------------------------------- per-bucket LDS aggregation
// One workgroup per hash bucket sums every record of its bucket -- the map workgroups' tail regions
// (count 1 each), the bucket's slice of every map workgroup's flushed LDS table and the bucket's
// overflow list -- in an LDS table.  A key that finds no slot within the probe limit (more distinct
// keys in the bucket than the table holds) goes to the overflow list; since slots only ever fill, a
// key that failed once fails always, so the LDS table and the overflow path never share a key.
//
// Throughput: the tail regions are the bulk (hundreds of MB); every wave streams them in chunks of
// 4 records per lane (1 KiB per load instruction), with the next chunk's loads in flight while the
// current one is summed, and a record that finds its key costs one 16-byte LDS read + one LDS add.
constexpr int BA_WG = 1024;
constexpr int BA_NW = BA_WG / 64;
// LDS table slots per bucket: wc with 32-bit counts (the job has fewer than 2^32 tokens) 6912
// (16-byte key + 4-byte count: 135 KiB, beside 16 KiB of miss queues), wc with 64-bit counts 6112
// (143 KiB), the indexer 4096 (+ 4-byte doc); the rest of the LDS holds the per-region record counts
// and chunk offsets.  More than half the slots stay free at 2^20 distinct keys over 256 buckets.
template <bool IDX, bool C32>
constexpr uint32_t ba_cap() { return IDX ? 4096u : (C32 ? 6912u : 6112u); }
constexpr int BA_PROBE = 64;
constexpr int BA_U = 8;            // records per lane per chunk
template <bool C32>
constexpr int ba_maxreg() { return C32 ? 512 : 2048; }  // map workgroups (regions) the size table holds
// wc with 32-bit counts: records whose first probe misses wait in a per-wave LDS queue of BA_QN and are
// probed a (nearly) full wave at a time
constexpr uint32_t BA_QN = 64;
template <bool IDX, bool C32>
constexpr bool ba_queue() { return !IDX && C32; }

#define GASK __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ GASK T *gk(T *p) {
    return (GASK T *)p;
}
typedef uint64_t u64x2k __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3k __attribute__((ext_vector_type(3), aligned(4)));  // a 12-byte wc tail record

// the map kernel's key hash (k_map.hip key_hash): bucket = top 9 bits
__device__ __forceinline__ uint32_t ba_hash(uint64_t a, uint64_t b, uint32_t d, uint32_t hash_bits) {
    uint32_t h = mrg_key_hash32(a, b, d);
    if (hash_bits && hash_bits < 32) h &= (1u << hash_bits) - 1u;
    return h;
}

struct alignas(16) BaKey {
    unsigned long long a, b;
};

// first probe slot of hash h: 16 hash bits below the bucket bits scaled to [0, CAP)
template <bool IDX, bool C32>
__device__ __forceinline__ uint32_t ba_slot(uint32_t h) {
    return (((h >> (32 - MRG_NBUCKET_LOG2 - 16)) & 0xFFFFu) * ba_cap<IDX, C32>()) >> 16;
}

// Add c to key (a, b[, d]).  Slots fill monotonically (k0, then k1, then doc, each by CAS from its
// empty value), so a slot whose fields all equal the key is the key's slot for good: the common case
// is one 16-byte read and one add.  A partly claimed slot is resolved by the CAS protocol.
// first: the key of the first probe slot, read by the caller (possibly before other adds: a stale
// EMPTY is resolved by the CAS protocol below, and a filled slot never changes)
template <bool IDX, bool C32, class CT>
__device__ __forceinline__ bool ba_add_from(BaKey *key, CT *cnt, unsigned int *doc, uint64_t a,
                                            uint64_t b, uint32_t d, uint64_t c, uint32_t h, BaKey first) {
    constexpr uint32_t CAP = ba_cap<IDX, C32>();
    uint32_t slot = ba_slot<IDX, C32>(h);
    BaKey kn = first;
    for (int p = 0; p < BA_PROBE; ++p) {
        const BaKey k = kn;
        // the next probe slot's key is read now, beside this one's processing (a stale EMPTY there is
        // resolved by the CAS below; a filled slot never changes)
        uint32_t nxt = slot + 1u + (uint32_t)p;  // triangular steps (one wrap at most: p < 64 <= CAP)
        if (nxt >= CAP) nxt -= CAP;
        kn = key[nxt];
        const bool dk = !IDX || doc[slot] == d;
        if (k.a == a && k.b == b && dk) {
            atomicAdd(&cnt[slot], (CT)c);
            return true;
        }
        if (k.a == MRG_EMPTY_K0 || (k.a == a && (k.b == MRG_EMPTY_K1 || (IDX && k.b == b)))) {
            const unsigned long long x = atomicCAS(&key[slot].a, MRG_EMPTY_K0, (unsigned long long)a);
            if (x == MRG_EMPTY_K0 || x == a) {
                const unsigned long long y = atomicCAS(&key[slot].b, MRG_EMPTY_K1, (unsigned long long)b);
                if (y == MRG_EMPTY_K1 || y == b) {
                    bool ok = true;
                    if (IDX) {
                        const unsigned int z = atomicCAS(&doc[slot], MRG_EMPTY_DOC, d);
                        ok = (z == MRG_EMPTY_DOC || z == d);
                    }
                    if (ok) {
                        atomicAdd(&cnt[slot], (CT)c);
                        return true;
                    }
                }
            }
        }
        slot = nxt;
    }
    return false;
}

template <bool IDX, bool C32, class CT>
__device__ __forceinline__ bool ba_add(BaKey *key, CT *cnt, unsigned int *doc, uint64_t a,
                                       uint64_t b, uint32_t d, uint64_t c, uint32_t h) {
    return ba_add_from<IDX, C32>(key, cnt, doc, a, b, d, c, h, key[ba_slot<IDX, C32>(h)]);
}

#ifndef MRG_AGG_XCD
#define MRG_AGG_XCD 1
#endif
static_assert(MRG_NBUCKET % 8 == 0, "buckets spread over the 8 XCDs");
template <bool IDX, bool C32>
__global__ __launch_bounds__(BA_WG, 1) void k_bucket_agg(BucketArgs A) {
    constexpr uint32_t BA_CAP = ba_cap<IDX, C32>();
    using CT = typename std::conditional<C32, unsigned int, unsigned long long>::type;
    __shared__ BaKey s_key[BA_CAP];
    __shared__ CT s_cnt[BA_CAP];
    __shared__ unsigned int s_doc[IDX ? BA_CAP : 1];
    __shared__ uint32_t s_rn[ba_maxreg<C32>()];      // tail records of region r in this bucket
    __shared__ uint32_t s_cs[ba_maxreg<C32>() + 1];  // first chunk of region r (chunks numbered region by region)
    __shared__ BaKey s_mq[ba_queue<IDX, C32>() ? BA_NW : 1][ba_queue<IDX, C32>() ? BA_QN : 1];  // miss queues
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < (int)BA_CAP; i += BA_WG) {
        s_key[i] = BaKey{MRG_EMPTY_K0, MRG_EMPTY_K1};
        s_cnt[i] = 0;
        if (IDX) s_doc[i] = MRG_EMPTY_DOC;
    }
    // workgroup (b, j): bucket b, hash sub-range j of A.nsub (a bucket with more distinct keys than one
    // table holds is summed by nsub workgroups, each reading all of its records and keeping its range)
    // With sub-ranges, the nsub workgroups of a bucket run side by side on ONE XCD (workgroups go to the
    // XCDs round-robin by blockIdx), so the second and third reads of the bucket's records come from
    // that XCD's L2 instead of HBM (MRG_AGG_XCD; 0 = bucket-major, the r05 order)
    const uint32_t nsub = A.nsub;
#if MRG_AGG_XCD
    const uint32_t g = blockIdx.x, slot = g / 8u;
    const uint32_t b = nsub > 1u ? (slot / nsub) * 8u + g % 8u : g % MRG_NBUCKET;
    const uint32_t jsub = nsub > 1u ? slot % nsub : g / MRG_NBUCKET;
#else
    const uint32_t b = blockIdx.x % MRG_NBUCKET, jsub = blockIdx.x / MRG_NBUCKET;
#endif
    auto mine = [&](uint32_t h) { return nsub <= 1u || (((h & 0xFFu) * nsub) >> 8) == jsub; };
    constexpr uint32_t RW = IDX ? 3u : 2u;
    const uint32_t cap = gk(A.bcap)[b];
    const uint32_t nreg = A.nreg;
    for (uint32_t r = tid; r < nreg; r += BA_WG) s_rn[r] = min(gk(A.bcount)[(uint64_t)r * MRG_NBUCKET + b], cap);
    __syncthreads();
    constexpr uint32_t CH = 64u * BA_U;  // records per chunk
    if (wv == 0) {  // chunk offsets of the regions: a wave scan, 64 regions at a time
        uint32_t run = 0;
        for (uint32_t r0 = 0; r0 < nreg; r0 += 64) {
            const uint32_t r = r0 + (uint32_t)lane;
            const uint32_t c = r < nreg ? (s_rn[r] + CH - 1u) / CH : 0u;
            uint32_t incl = c;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            if (r < nreg) s_cs[r] = run + incl - c;
            run += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        if (lane == 0) s_cs[nreg] = run;
    }
    __syncthreads();
    const uint32_t NC = s_cs[nreg];  // chunks of the bucket

    auto overflow = [&](bool ovf, uint64_t a, uint64_t c, uint32_t d, uint64_t n2) {
        const uint64_t j = mrg_wave_append(&A.counters[CNT_OVF2], ovf);
        if (ovf && j < A.ocap) {
            gk(A.ok0)[j] = a; gk(A.ok1)[j] = c; gk(A.ocnt)[j] = (uint32_t)n2;
            if (IDX) gk(A.odoc)[j] = d;
        }
    };

    // ---- 1. tail regions, as one sequence of chunks of 64 * BA_U records (region by region): wave wv
    // takes chunks wv, wv + 16, ..., so at any time the workgroup's 16 waves read 16 neighbouring chunks
    // (one stream of the bucket per workgroup; with a region per wave the 256 workgroups kept 4096
    // streams open at once)
    // the bucket's regions: 12-byte records (wc) / 24-byte records (indexer)
    const GASK uint8_t *pool = reinterpret_cast<const GASK uint8_t *>(gk(A.pool)) + A.rbase[b] * MRG_TAIL_BYTES(IDX);
    struct Chunk {
        u64x2k k[BA_U];
        uint32_t d[IDX ? BA_U : 1];
    };
    // region and record offset of chunk k (r only moves forward: a wave's chunks increase)
    auto chunk_pos = [&](uint32_t k, uint32_t &r) -> uint32_t {
        while (s_cs[r + 1] <= k) ++r;
        return (k - s_cs[r]) * CH;
    };
    // unconditional loads: an index past the region's end reads its last record (masked later)
    auto load_chunk = [&](uint32_t r, uint32_t off, Chunk &X) {
        const uint32_t n = s_rn[r];
        const GASK uint8_t *src = pool + (uint64_t)r * cap * MRG_TAIL_BYTES(IDX);
#pragma unroll
        for (int k = 0; k < BA_U; ++k) {
            const uint32_t i = min(off + 64u * k + (uint32_t)lane, n - 1u);
            if (IDX) {
                const GASK uint64_t *rec = reinterpret_cast<const GASK uint64_t *>(src) + (uint64_t)i * 3;
                X.k[k] = u64x2k{rec[0], rec[1]};
                X.d[k] = (uint32_t)rec[2];
            } else {
                // read once: non-temporal (A/B: aggregation -1.5 %); {k0, high word of k1}
                const u32x3k v = __builtin_nontemporal_load(reinterpret_cast<const GASK u32x3k *>(src + (uint64_t)i * 12u));
                X.k[k] = u64x2k{(uint64_t)v.x | ((uint64_t)v.y << 32), (uint64_t)v.z << 32};
            }
        }
    };
    auto settle = [](Chunk &X) {
#pragma unroll
        for (int k = 0; k < BA_U; ++k) asm volatile("" : "+v"(X.k[k]));
        if (IDX)
            for (int k = 0; k < BA_U; ++k) asm volatile("" : "+v"(X.d[k]));
    };
    uint64_t abl_acc = 0;  // MRG_AGG_ABLATE (timing only): what the skipped work would have consumed
    uint32_t qn = 0;       // records in this wave's miss queue (wave-uniform)
    auto drain = [&]() {   // the queued records, one per lane, through the full probe
        if (!ba_queue<IDX, C32>() || qn == 0) return;
        const bool act = (uint32_t)lane < qn;
        const BaKey r = s_mq[ba_queue<IDX, C32>() ? wv : 0][act ? lane : 0];
        bool ovf = false;
        if (act) {
            const uint32_t h = ba_hash(r.a, r.b, MRG_EMPTY_DOC, A.hash_bits);
            ovf = !ba_add<IDX, C32>(s_key, s_cnt, s_doc, r.a, r.b, MRG_EMPTY_DOC, 1ull, h);
        }
        if (__any(ovf)) overflow(ovf, r.a, r.b, MRG_EMPTY_DOC, 1);
        qn = 0;
    };
    // records of a chunk: every hash first, then record k + 1's first probe slot is read while
    // record k is added, so the probe chains of neighbouring records overlap by one LDS round trip
    auto sum_chunk = [&](uint32_t r, uint32_t off, const Chunk &X) {
        const uint32_t n = s_rn[r];
        if (A.ablate) {
#pragma unroll
            for (int k = 0; k < BA_U; ++k) {
                const bool ok = off + 64u * k + (uint32_t)lane < n;
                const uint64_t a = X.k[k].x, c = X.k[k].y;
                const uint32_t d = IDX ? X.d[k] : MRG_EMPTY_DOC;
                abl_acc += ok ? ((A.ablate & 2u) ? (a ^ c) : (uint64_t)ba_hash(a, c, d, A.hash_bits)) : 0u;
            }
            return;
        }
        uint32_t hk[BA_U];
#pragma unroll
        for (int k = 0; k < BA_U; ++k) hk[k] = ba_hash(X.k[k].x, X.k[k].y, IDX ? X.d[k] : MRG_EMPTY_DOC, A.hash_bits);
        BaKey pre = s_key[ba_slot<IDX, C32>(hk[0])];
        if constexpr (ba_queue<IDX, C32>()) {
            // first probe here (the key sits in its first slot: add); every other record joins the
            // wave's miss queue, which is probed when the next batch would overflow it
#pragma unroll
            for (int k = 0; k < BA_U; ++k) {
                const bool ok = off + 64u * k + (uint32_t)lane < n;
                const uint64_t a = X.k[k].x, c = X.k[k].y;
                const BaKey first = pre;
                if (k + 1 < BA_U) pre = s_key[ba_slot<IDX, C32>(hk[k + 1 < BA_U ? k + 1 : k])];
                const uint32_t h = hk[k];
                const bool me = ok && mine(h);
                const bool hit = me && first.a == a && first.b == c;
                if (hit) atomicAdd(&s_cnt[ba_slot<IDX, C32>(h)], (CT)1);
                const bool miss = me && !hit;
                const uint64_t mm = __ballot(miss);
                if (mm) {
                    const uint32_t m = (uint32_t)__builtin_popcountll(mm);
                    if (qn + m > BA_QN) drain();
                    if (miss) s_mq[wv][qn + (uint32_t)__builtin_popcountll(mm & mrg_lanemask_lt())] = BaKey{a, c};
                    qn += m;
                }
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < BA_U; ++k) {
            const bool ok = off + 64u * k + (uint32_t)lane < n;
            const uint64_t a = X.k[k].x, c = X.k[k].y;
            const uint32_t d = IDX ? X.d[k] : MRG_EMPTY_DOC;
            const BaKey first = pre;
            if (k + 1 < BA_U) pre = s_key[ba_slot<IDX, C32>(hk[k + 1 < BA_U ? k + 1 : k])];
            bool ovf = false;
            const uint32_t h = hk[k];
            if (ok && mine(h)) ovf = !ba_add_from<IDX, C32>(s_key, s_cnt, s_doc, a, c, d, 1ull, h, first);
            if (__any(ovf)) overflow(ovf, a, c, d, 1);
        }
    };
    if (!(A.ablate & 4u)) {
        Chunk XA, XB;
        uint32_t kA = (uint32_t)wv, rA = 0, oA = 0;
        if (kA < NC) {
            oA = chunk_pos(kA, rA);
            load_chunk(rA, oA, XA);
        }
        while (kA < NC) {
            const uint32_t kB = kA + BA_NW;
            uint32_t rB = rA, oB = oA;
            if (kB < NC) oB = chunk_pos(kB, rB);
            settle(XA);
            load_chunk(rB, oB, XB);  // past the end: a reload of chunk kA (fixed load count)
            sum_chunk(rA, oA, XA);
            if (kB >= NC) break;
            kA = kB + BA_NW;
            rA = rB;
            if (kA < NC) oA = chunk_pos(kA, rA);
            else oA = oB;
            settle(XB);
            load_chunk(rA, oA, XA);
            sum_chunk(rB, oB, XB);
        }
    }
    drain();  // the rest of the miss queue

    if (A.ablate && abl_acc == 0x9E3779B97F4A7C15ull) atomicAdd(&A.counters[CNT_OVF2], 1ull);
    // ---- 2. this bucket's slice of every map workgroup's flushed table (a few entries each): the
    // wave's regions (wv, wv + 16, ...) one per lane, their slices flattened over the lanes (an
    // exclusive scan of the slice sizes, each entry finds its region by binary search), four entries
    // per lane in flight -- two load latencies per 64 regions instead of two per region
    {
        const uint32_t nrw = nreg > (uint32_t)wv ? (nreg - (uint32_t)wv + BA_NW - 1) / BA_NW : 0u;
        for (uint32_t l0 = 0; l0 < nrw; l0 += 64) {
            const uint32_t l = l0 + (uint32_t)lane;
            uint32_t lo = 0, cnt = 0;
            if (l < nrw) {
                const GASK uint32_t *fo = gk(A.foff) + (uint64_t)(wv + BA_NW * l) * (MRG_NBUCKET + 1);
                lo = fo[b];
                cnt = fo[b + 1] - lo;
            }
            uint32_t incl = cnt;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(incl, o);
                if (lane >= o) incl += v;
            }
            const uint32_t excl = incl - cnt;
            const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            for (uint32_t e0 = 0; e0 < total; e0 += 256) {
                uint64_t a[4], c[4];
                uint32_t n2[4], d[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t e = e0 + 64u * u + (uint32_t)lane;
                    ok[u] = e < total;
                    uint32_t k = 0;  // last lane whose slice starts at or before e
#pragma unroll
                    for (int st = 32; st > 0; st >>= 1)
                        if (__shfl(excl, (int)(k + st)) <= e) k += st;
                    const uint32_t rl = l0 + k;
                    const uint64_t at = (uint64_t)(wv + BA_NW * rl) * A.regcap + __shfl(lo, (int)k) + (e - __shfl(excl, (int)k));
                    a[u] = 0; c[u] = 0; n2[u] = 0; d[u] = MRG_EMPTY_DOC;
                    if (ok[u]) {
                        a[u] = gk(A.fk0)[at];
                        c[u] = gk(A.fk1)[at];
                        n2[u] = gk(A.fcnt)[at];
                        if (IDX) d[u] = gk(A.fdoc)[at];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    bool ovf = false;
                    if (ok[u]) {
                        const uint32_t h = ba_hash(a[u], c[u], d[u], A.hash_bits);
                        if (mine(h)) ovf = !ba_add<IDX, C32>(s_key, s_cnt, s_doc, a[u], c[u], d[u], n2[u], h);
                    }
                    if (__any(ovf)) overflow(ovf, a[u], c[u], d[u], n2[u]);
                }
            }
        }
    }
    // ---- 3a. wc keys of 13..16 bytes: the bucket's 16-byte regions, wave wv taking regions wv, wv + 16, ..
    if (!IDX) {
        const uint32_t cap16 = gk(A.bcap16)[b];
        const GASK uint64_t *p16 = gk(A.pool16) + 2ull * A.rbase16[b];
        for (uint32_t r = (uint32_t)wv; r < nreg; r += BA_NW) {
            const uint32_t n = min(gk(A.bcount16)[(uint64_t)r * MRG_NBUCKET + b], cap16);
            const GASK uint64_t *src = p16 + 2ull * r * cap16;
            for (uint32_t base = 0; base < n; base += 64) {
                const uint32_t i = base + (uint32_t)lane;
                bool ovf = false;
                uint64_t a = 0, c = 0;
                if (i < n) {
                    const u64x2k v = *reinterpret_cast<const GASK u64x2k *>(src + 2ull * i);
                    a = v.x;
                    c = v.y;
                    const uint32_t h = ba_hash(a, c, MRG_EMPTY_DOC, A.hash_bits);
                    if (mine(h)) ovf = !ba_add<IDX, C32>(s_key, s_cnt, s_doc, a, c, MRG_EMPTY_DOC, 1ull, h);
                }
                if (__any(ovf)) overflow(ovf, a, c, MRG_EMPTY_DOC, 1);
            }
        }
    }
    // ---- 3. records that did not fit their map workgroup's region: this bucket's overflow list
    {
        const uint32_t n = min(gk(A.monext)[b], A.mocap);
        const GASK uint64_t *src = gk(A.movf) + (uint64_t)b * A.mocap * RW;
        for (uint32_t base = wv * 64u; base < n; base += BA_WG) {
            const uint32_t i = base + lane;
            bool ovf = false;
            uint64_t a = 0, c = 0;
            uint32_t d = MRG_EMPTY_DOC;
            if (i < n) {
                a = src[(uint64_t)i * RW];
                c = src[(uint64_t)i * RW + 1];
                if (IDX) d = (uint32_t)src[(uint64_t)i * RW + 2];
                const uint32_t h = ba_hash(a, c, d, A.hash_bits);
                if (mine(h)) ovf = !ba_add<IDX, C32>(s_key, s_cnt, s_doc, a, c, d, 1ull, h);
            }
            if (__any(ovf)) overflow(ovf, a, c, d, 1);
        }
    }
    __syncthreads();
    // the keys out: per-wave counts of every pass of 1024 slots in one sweep, one wave scan, ONE
    // device atomic per workgroup (was one per pass: 1792 on one counter at the end of the launch)
    constexpr int NP = (int)((BA_CAP + BA_WG - 1) / BA_WG);
    constexpr int NPW = NP * BA_NW;
    static_assert(NPW <= 128, "one wave scans two entries per lane");
    __shared__ uint32_t s_po[NPW];
    __shared__ unsigned long long s_base;
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
        const int i = pp * BA_WG + tid;
        const uint64_t m = __ballot(i < (int)BA_CAP && s_key[min(i, (int)BA_CAP - 1)].a != MRG_EMPTY_K0);
        if (lane == 0) s_po[pp * BA_NW + wv] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (wv == 0) {
        const int e0 = 2 * lane, e1 = e0 + 1;
        const uint32_t c0 = e0 < NPW ? s_po[e0] : 0u, c1 = e1 < NPW ? s_po[e1] : 0u;
        uint32_t incl = c0 + c1;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o);
            if (lane >= o) incl += v;
        }
        const uint32_t ex = incl - c0 - c1;
        if (e0 < NPW) s_po[e0] = ex;
        if (e1 < NPW) s_po[e1] = ex + c0;
        const uint32_t tot = (uint32_t)__shfl((int)incl, 63);
        if (lane == 0) s_base = tot ? atomicAdd(&A.counters[CNT_KEYS], (unsigned long long)tot) : 0ull;
    }
    __syncthreads();
    const uint64_t kbase = s_base;
    for (int pp = 0; pp < NP; ++pp) {
        const int i = min(pp * BA_WG + tid, (int)BA_CAP - 1);
        const BaKey k = s_key[i];
        const bool full = pp * BA_WG + tid < (int)BA_CAP && k.a != MRG_EMPTY_K0;
        const uint64_t m = __ballot(full);
        const uint64_t j = kbase + s_po[pp * BA_NW + wv] + (uint64_t)__popcll(m & mrg_lanemask_lt());
        if (full && j < A.kcap) {
            gk(A.out.k0)[j] = k.a;
            gk(A.out.k1)[j] = k.b;
            gk(A.out.cnt)[j] = s_cnt[i];
            gk(A.out.doc)[j] = IDX ? s_doc[i] : MRG_EMPTY_DOC;
            const uint32_t L = mrg_short_len(k.a, k.b);
            gk(A.out.len)[j] = L;
            gk(A.out.hoff)[j] = MRG_NO_HEAP;
            // the partition right here (worker.rs:129), instead of a k_partition pass over the keys
            if (A.n_reduce) gk(A.out.part)[j] = (uint32_t)(mrg_siphash_short(k.a, k.b, L) % (uint64_t)A.n_reduce);
        }
    }
}

// the staged small writes of a job's setup (mrg_internal.h StageOp), in their issue order -- one
// workgroup, a barrier between writes: a batch may write a range twice (zero the counters, then set
// one of them to ~0), and the later write must win, as it did as separate stream operations
__global__ __launch_bounds__(1024) void k_stage_scatter(const uint8_t *stage, uint32_t table_off, uint32_t nops) {
    const StageOp *ops = reinterpret_cast<const StageOp *>(stage + table_off);
    for (uint32_t k = 0; k < nops; ++k) {
        const StageOp op = ops[k];
        uint8_t *dst = reinterpret_cast<uint8_t *>(op.dst);
        const bool fill = op.src == 0xFFFFFFFFu;
        if (((op.dst | op.n) & 3u) == 0u) {  // dword aligned (every pool block and staging offset is)
            const uint32_t f4 = op.fill * 0x01010101u;
            const uint32_t *src = reinterpret_cast<const uint32_t *>(stage + (fill ? 0u : op.src));
            for (uint32_t i = threadIdx.x; i < op.n / 4u; i += blockDim.x)
                reinterpret_cast<uint32_t *>(dst)[i] = fill ? f4 : src[i];
        } else {
            for (uint32_t i = threadIdx.x; i < op.n; i += blockDim.x) dst[i] = fill ? (uint8_t)op.fill : stage[op.src + i];
        }
        __syncthreads();  // (global writes of this workgroup: ordered by the barrier's release)
    }
}

__global__ void k_table_clear(TableArgs T, bool idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T.cap) return;
    T.tk0[i] = MRG_EMPTY_K0;
    T.tk1[i] = MRG_EMPTY_K1;
    T.tcnt[i] = 0;
    if (idx) T.tdoc[i] = MRG_EMPTY_DOC;
}

__device__ __forceinline__ void table_add(const TableArgs &T, uint64_t a, uint64_t b, uint32_t d, uint64_t c,
                                          bool idx) {
    uint64_t h = mrg_key_mix(a, b, d);
    if (T.hash_bits) h &= (1ull << T.hash_bits) - 1u;
    uint64_t slot = (h ^ (h >> 31)) & (T.cap - 1);
    for (uint64_t probe = 0; probe < T.cap; ++probe) {
        const unsigned long long x =
            atomicCAS((unsigned long long *)&T.tk0[slot], MRG_EMPTY_K0, (unsigned long long)a);
        if (x == MRG_EMPTY_K0 || x == a) {
            const unsigned long long y =
                atomicCAS((unsigned long long *)&T.tk1[slot], MRG_EMPTY_K1, (unsigned long long)b);
            if (y == MRG_EMPTY_K1 || y == b) {
                bool ok = true;
                if (idx) {
                    const unsigned int z = atomicCAS(&T.tdoc[slot], MRG_EMPTY_DOC, d);
                    ok = (z == MRG_EMPTY_DOC || z == d);
                }
                if (ok) {
                    atomicAdd((unsigned long long *)&T.tcnt[slot], (unsigned long long)c);
                    return;
                }
            }
        }
        // triangular steps (+1, +2, +3, ...: every slot of the power-of-two table is reached): no
        // primary clusters, so few probes even when the hash values crowd into part of the table
        // (the collision test knob truncates them to 20 bits while the table has more slots)
        slot = (slot + probe + 1u) & (T.cap - 1);
    }
}

__global__ void k_table_insert(TableArgs T, const uint64_t *k0, const uint64_t *k1, const uint32_t *cnt,
                               const uint32_t *doc, uint64_t n, bool idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    table_add(T, k0[i], k1[i], idx ? doc[i] : MRG_EMPTY_DOC, cnt[i], idx);
}

// short exchange records (include/mrgpu.h): v = count (wc) / doc id (indexer)
__global__ void k_table_insert_x(TableArgs T, const XRec *x, uint64_t n, bool idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const XRec r = x[i];
    if (r.len > 16u) return;  // long keys take the fingerprint-sort path
    table_add(T, r.a, r.b, idx ? r.v : MRG_EMPTY_DOC, idx ? 1ull : (uint64_t)r.v, idx);
}

__global__ void k_table_insert_l(TableArgs T, const LRec *x, uint64_t n, bool idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const LRec r = x[i];
    if (r.len > 16u) return;
    table_add(T, r.k0, r.k1, idx ? r.doc : MRG_EMPTY_DOC, r.cnt, idx);
}

constexpr int TC_WG = 1024;
__global__ __launch_bounds__(TC_WG) void k_table_compact(TableArgs T, bool idx, KeySet out, unsigned long long *counter) {
    __shared__ uint32_t s_w[TC_WG / 64];
    __shared__ unsigned long long s_base;
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool full = i < T.cap && T.tk0[i] != MRG_EMPTY_K0;
    const uint64_t j = wg_append<TC_WG>(counter, full, s_w, &s_base);
    if (!full) return;
    const uint64_t a = T.tk0[i], b = T.tk1[i];
    out.k0[j] = a;
    out.k1[j] = b;
    out.cnt[j] = T.tcnt[i];
    out.doc[j] = idx ? T.tdoc[i] : MRG_EMPTY_DOC;
    out.len[j] = mrg_short_len(a, b);
    out.hoff[j] = MRG_NO_HEAP;
}

// worker.rs:129  index = (DefaultHasher(key) % reduce_n as u64) as i32
__global__ void k_partition(KeySet ks, const uint8_t *heap, uint64_t n, uint32_t n_reduce) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t L = ks.len[i];
    const uint64_t h = L <= 16u ? mrg_siphash_short(ks.k0[i], ks.k1[i], L) : mrg_siphash_bytes(heap + ks.hoff[i], L);
    ks.part[i] = (uint32_t)(h % (uint64_t)n_reduce);
}

// ---------------------------------------------------------------- wide (sort-based) aggregation
// High-cardinality inputs (~1e9 near-unique keys): almost every token misses the
// map-side combine and no per-bucket LDS table can hold a bucket's keys, so instead of hashing, every
// map record (tail regions, flushed tables, overflow lists) is gathered as a sort record with its
// partition (SipHash-1-3 % nReduce, worker.rs:111-115, 129) and count, sorted by (partition, key),
// and equal keys are summed by a segmented scan.  The key set then comes out in output order, so the
// reduce-side sort (worker.rs:162-164) is skipped.  wc only (no doc component).
//
// Segments: [nreg * NB tail regions (12-byte records), s = b * nreg + w] [nreg flush regions]
// [NB overflow lists] [nreg * NB 16-byte tail regions].
__global__ void k_wide_counts(BucketArgs A, uint64_t *cnt) {
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t nt = (uint64_t)A.nreg * MRG_NBUCKET;
    if (s < nt) {
        const uint32_t b = (uint32_t)(s / A.nreg), w = (uint32_t)(s % A.nreg);
        cnt[s] = min(A.bcount[(uint64_t)w * MRG_NBUCKET + b], A.bcap[b]);
    } else if (s < nt + A.nreg) {
        const uint64_t w = s - nt;
        cnt[s] = A.foff[w * (MRG_NBUCKET + 1) + MRG_NBUCKET];
    } else if (s < nt + A.nreg + MRG_NBUCKET) {
        const uint32_t b = (uint32_t)(s - nt - A.nreg);
        cnt[s] = min(A.monext[b], A.mocap);
    } else if (s < 2 * nt + A.nreg + MRG_NBUCKET) {
        const uint64_t s2 = s - nt - A.nreg - MRG_NBUCKET;
        const uint32_t b = (uint32_t)(s2 / A.nreg), w = (uint32_t)(s2 % A.nreg);
        cnt[s] = min(A.bcount16[(uint64_t)w * MRG_NBUCKET + b], A.bcap16[b]);
    }
}

// one workgroup per segment; record -> SortRec{k0, k1, part, doc = 0, idx = count}
__global__ void k_wide_gather(BucketArgs A, const uint64_t *off, uint32_t n_reduce, SortRec *out) {
    const uint64_t s = blockIdx.x;
    const uint64_t nt = (uint64_t)A.nreg * MRG_NBUCKET;
    const uint64_t o = off[s], n = off[s + 1] - o;
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        uint64_t k0, k1;
        uint32_t c = 1;
        if (s < nt) {
            const uint32_t b = (uint32_t)(s / A.nreg), w = (uint32_t)(s % A.nreg);
            const uint64_t j = A.rbase[b] + (uint64_t)w * A.bcap[b] + i;
            const uint32_t *rec = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(A.pool) + 12u * j);
            k0 = (uint64_t)rec[0] | ((uint64_t)rec[1] << 32);
            k1 = (uint64_t)rec[2] << 32;
        } else if (s >= nt + A.nreg + MRG_NBUCKET) {
            const uint64_t s2 = s - nt - A.nreg - MRG_NBUCKET;
            const uint32_t b = (uint32_t)(s2 / A.nreg), w = (uint32_t)(s2 % A.nreg);
            const uint64_t j = A.rbase16[b] + (uint64_t)w * A.bcap16[b] + i;
            k0 = A.pool16[2 * j];
            k1 = A.pool16[2 * j + 1];
        } else if (s < nt + A.nreg) {
            const uint64_t j = (s - nt) * A.regcap + i;
            k0 = A.fk0[j];
            k1 = A.fk1[j];
            c = A.fcnt[j];
        } else {
            const uint64_t b = s - nt - A.nreg;
            const uint64_t j = b * A.mocap + i;
            k0 = A.movf[2 * j];
            k1 = A.movf[2 * j + 1];
        }
        SortRec r;
        r.k0 = k0;
        r.k1 = k1;
        r.part = (uint32_t)(mrg_siphash_short(k0, k1, mrg_short_len(k0, k1)) % (uint64_t)n_reduce);
        r.doc = 0;
        r.idx = c;
        r.pad = 0;
        out[o + i] = r;
    }
}

__global__ void k_wide_heads(const SortRec *r, uint64_t n, uint64_t *head, uint64_t *cv) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    head[i] = (i == 0 || r[i].k0 != r[i - 1].k0 || r[i].k1 != r[i - 1].k1) ? 1u : 0u;  // part follows the key
    cv[i] = r[i].idx;
}

// E = exclusive scan of head (run index), C = exclusive scan of counts.  The head of run k writes
// the key and F[k] = its first record.
__global__ void k_wide_keys(const SortRec *r, uint64_t n, const uint64_t *head, const uint64_t *E, KeySet ks,
                            uint64_t *F) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !head[i]) return;
    const uint64_t k = E[i];
    ks.k0[k] = r[i].k0;
    ks.k1[k] = r[i].k1;
    ks.doc[k] = MRG_EMPTY_DOC;
    ks.len[k] = mrg_short_len(r[i].k0, r[i].k1);
    ks.part[k] = r[i].part;
    ks.hoff[k] = MRG_NO_HEAP;
    F[k] = i;
}

// count of run k = sum of the counts of its records (C[end] - C[first], C[n] = total)
__global__ void k_wide_cnt(const uint64_t *F, uint64_t runs, uint64_t n, const uint64_t *C, uint64_t ctot, KeySet ks) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= runs) return;
    const uint64_t e = k + 1 < runs ? C[F[k + 1]] : ctot;
    ks.cnt[k] = e - C[F[k]];
}

// Long keys after the fingerprint sort: element i (sorted order) belongs to the run of equal
// fingerprints; within the run its representative is the FIRST element with equal full key bytes
// (and doc): the collision-safe tie-break, equal fingerprints never merge different strings.
__global__ void k_long_group(const uint64_t *fp, const uint32_t *idx, const uint32_t *doc, const uint8_t *heap,
                             const uint64_t *hoff, const uint32_t *flen, uint64_t n, uint32_t *rep) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t me = idx[i];
    const uint64_t f = fp[i];
    uint64_t g = 0, hi = i;  // first index of the run of fingerprint f
    while (g < hi) {
        const uint64_t mid = (g + hi) >> 1;
        if (fp[mid] < f) g = mid + 1; else hi = mid;
    }
    uint32_t r = me;
    const uint8_t *mk = heap + hoff[me];
    const uint32_t ml = flen[me];
    for (uint64_t j = g; j < i; ++j) {
        const uint32_t o = idx[j];
        if (flen[o] != ml || (doc && doc[o] != doc[me])) continue;
        const uint8_t *ok = heap + hoff[o];
        bool eq = true;
        for (uint32_t b = 0; b < ml && eq; ++b) eq = mk[b] == ok[b];
        if (eq) { r = o; break; }
    }
    rep[me] = r;
}

__global__ void k_long_count(const uint32_t *rep, const uint64_t *cnt_in, uint64_t n, unsigned long long *acc) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    atomicAdd(&acc[rep[i]], (unsigned long long)(cnt_in ? cnt_in[i] : 1u));
}

__global__ void k_long_emit(const uint32_t *rep, const uint64_t *k0, const uint64_t *k1, const uint32_t *flen,
                            const uint64_t *hoff, const uint32_t *doc, uint64_t n, const unsigned long long *acc,
                            KeySet out, unsigned long long *counter, bool idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool mine = i < n && rep[i] == (uint32_t)i;
    const uint64_t j = mrg_wave_append(counter, mine);
    if (!mine) return;
    out.k0[j] = k0[i];
    out.k1[j] = k1[i];
    out.cnt[j] = acc[i];
    out.doc[j] = idx ? doc[i] : MRG_EMPTY_DOC;
    out.len[j] = flen[i];
    out.hoff[j] = hoff[i];
}

// segment (sender) of record i: the first s with i < seg_rec_end[s] (binary search)
__device__ __forceinline__ uint32_t seg_of(const uint64_t *seg_rec_end, uint32_t n_segs, uint64_t i) {
    uint32_t lo = 0, hi = n_segs - 1u;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (i < seg_rec_end[mid]) hi = mid;
        else lo = mid + 1u;
    }
    return lo;
}

// received exchange records with long keys -> long items over the received heap (long form: a = heap
// offset in the sender's segment, b = count, v = doc)
__global__ void k_x_split_long(const XRec *x, uint64_t n, const uint64_t *seg_rec_end, const uint64_t *seg_heap_base,
                               uint32_t n_segs, LongItems li, unsigned long long *counter, bool idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool lng = i < n && x[i].len > 16u;
    const uint64_t j = mrg_wave_append(counter, lng);
    if (!lng) return;
    const XRec r = x[i];
    li.start[j] = seg_heap_base[seg_of(seg_rec_end, n_segs, i)] + r.a;
    li.rawlen[j] = r.len;
    li.doc[j] = idx ? r.v : MRG_EMPTY_DOC;
    li.cnt[j] = idx ? 1ull : r.b;
}

// the same for the text reduce's line records (key bytes addressed in their file's segment)
__global__ void k_l_split_long(const LRec *x, uint64_t n, const uint64_t *seg_rec_end, const uint64_t *seg_heap_base,
                               uint32_t n_segs, LongItems li, unsigned long long *counter) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool lng = i < n && x[i].len > 16u;
    const uint64_t j = mrg_wave_append(counter, lng);
    if (!lng) return;
    const LRec r = x[i];
    li.start[j] = seg_heap_base[seg_of(seg_rec_end, n_segs, i)] + r.heap;
    li.rawlen[j] = r.len;
    li.doc[j] = r.doc;
    li.cnt[j] = r.cnt;
}

// Export of the distinct keys by owner (part % n_owners).  Every workgroup counts its keys per owner
// in LDS and takes its ranges with one device atomic per owner (a device atomic per key on n_owners
// addresses serialised: 12.6 ms per 1 M keys for one owner); more owners than EXP_MAXO fall back to
// per-key atomics.
constexpr int EXP_WG = 1024;
constexpr uint32_t EXP_MAXO = 256;

__global__ __launch_bounds__(EXP_WG) void k_export_count(KeySet ks, uint64_t n, uint32_t n_owners,
                                                         unsigned long long *rec_cnt, unsigned long long *heap_cnt,
                                                         bool idx, uint64_t vmax) {
    __shared__ unsigned long long s_rc[EXP_MAXO];
    __shared__ unsigned long long s_hc[EXP_MAXO];
    const bool lds = n_owners <= EXP_MAXO;
    if (lds)
        for (uint32_t o = threadIdx.x; o < n_owners; o += EXP_WG) {
            s_rc[o] = 0;
            s_hc[o] = 0;
        }
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t o = ks.part[i] % n_owners;
        const uint32_t len = ks.len[i];
        const unsigned long long nr = mrg_xrec_per_key(ks.cnt[i], len, idx, vmax);
        if (lds) {
            atomicAdd(&s_rc[o], nr);
            if (len > 16u) atomicAdd(&s_hc[o], (unsigned long long)len);
        } else {
            atomicAdd(&rec_cnt[o], nr);
            if (len > 16u) atomicAdd(&heap_cnt[o], (unsigned long long)len);
        }
    }
    if (!lds) return;
    __syncthreads();
    for (uint32_t o = threadIdx.x; o < n_owners; o += EXP_WG) {
        if (s_rc[o]) atomicAdd(&rec_cnt[o], (unsigned long long)s_rc[o]);
        if (s_hc[o]) atomicAdd(&heap_cnt[o], s_hc[o]);
    }
}

__global__ __launch_bounds__(EXP_WG) void k_export_pack(KeySet ks, const uint8_t *heap, uint64_t n, uint32_t n_owners,
                                                        const uint64_t *rec_base, const uint64_t *heap_base,
                                                        unsigned long long *rec_cur, unsigned long long *heap_cur,
                                                        XRec *out, uint8_t *out_heap, bool idx, uint64_t vmax) {
    __shared__ unsigned long long s_rc[EXP_MAXO];
    __shared__ unsigned long long s_hc[EXP_MAXO], s_rb[EXP_MAXO], s_hb[EXP_MAXO];
    const bool lds = n_owners <= EXP_MAXO;
    if (lds)
        for (uint32_t o = threadIdx.x; o < n_owners; o += EXP_WG) {
            s_rc[o] = 0;
            s_hc[o] = 0;
        }
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = i < n;
    uint32_t o = 0, len = 0;
    uint64_t cnt = 0, nr = 0;
    unsigned long long lr = 0, lh = 0;  // this key's rank / heap offset inside the workgroup's range
    if (act) {
        o = ks.part[i] % n_owners;
        len = ks.len[i];
        cnt = ks.cnt[i];
        nr = mrg_xrec_per_key(cnt, len, idx, vmax);
        if (lds) {
            lr = atomicAdd(&s_rc[o], (unsigned long long)nr);
            if (len > 16u) lh = atomicAdd(&s_hc[o], (unsigned long long)len);
        } else {
            lr = atomicAdd(&rec_cur[o], (unsigned long long)nr);
            if (len > 16u) lh = atomicAdd(&heap_cur[o], (unsigned long long)len);
        }
    }
    if (lds) {
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < n_owners; q += EXP_WG) {
            s_rb[q] = s_rc[q] ? atomicAdd(&rec_cur[q], (unsigned long long)s_rc[q]) : 0ull;
            s_hb[q] = s_hc[q] ? atomicAdd(&heap_cur[q], s_hc[q]) : 0ull;
        }
        __syncthreads();
        if (act) {
            lr += s_rb[o];
            lh += s_hb[o];
        }
    }
    if (!act) return;
    const uint64_t slot = rec_base[o] + lr;
    XRec r;
    r.len = len;
    if (len > 16u) {  // long form: heap offset relative to the owner's segment, 64-bit count
        const uint8_t *src = heap + ks.hoff[i];
        uint8_t *dst = out_heap + heap_base[o] + lh;
        for (uint32_t b = 0; b < len; ++b) dst[b] = src[b];
        r.a = lh;
        r.b = idx ? 1ull : cnt;
        r.v = idx ? ks.doc[i] : MRG_EMPTY_DOC;
        out[slot] = r;
        return;
    }
    r.a = ks.k0[i];
    r.b = ks.k1[i];
    if (idx) {
        r.v = ks.doc[i];
        out[slot] = r;
        return;
    }
    for (uint64_t k = 0; k < nr; ++k) {  // counts above 32 bits: several records, summed by the receiver
        const uint64_t c = cnt > vmax ? vmax : cnt;
        cnt -= c;
        r.v = (uint32_t)c;
        out[slot + k] = r;
    }
}

// carry (wc): the key's count and length ride in the record (doc = count bits 0..31, pad = length
// (0xFF: a long key, length in the key set) | count bits 32..55 << 8), so the formatter reads each
// sorted record once instead of gathering len / cnt from the key set twice.  (wc keys are distinct:
// doc only orders long keys with equal 16-byte prefixes, which k_fix_runs orders by full bytes.)
__global__ void k_make_sortrec(KeySet ks, uint64_t n, const uint32_t *doc_rank, SortRec *out, int carry) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SortRec r;
    r.k0 = ks.k0[i];
    r.k1 = ks.k1[i];
    r.part = ks.part[i];
    r.doc = doc_rank ? doc_rank[ks.doc[i]] : 0u;
    r.idx = (uint32_t)i;
    r.pad = 0;
    if (carry) {
        const uint64_t c = ks.cnt[i];
        const uint32_t len = ks.len[i];
        r.doc = (uint32_t)c;
        r.pad = (len <= 16u ? len : 0xFFu) | ((uint32_t)(c >> 32) << 8);
    }
    out[i] = r;
}

template <class T>
__global__ void k_fill(T *p, T v, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}
__global__ void k_iota(uint32_t *p, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}

}  // namespace

void mrg_launch_stage_scatter(const uint8_t *d_stage, uint32_t table_off, uint32_t nops, hipStream_t s) {
    if (nops) hipLaunchKernelGGL(k_stage_scatter, dim3(1), dim3(1024), 0, s, d_stage, table_off, nops);
}

void mrg_launch_bucket_agg(const BucketArgs &a, bool indexer, bool count32, hipStream_t s) {
    const dim3 g(MRG_NBUCKET * std::max<uint32_t>(a.nsub, 1u));
    if (indexer) hipLaunchKernelGGL((k_bucket_agg<true, false>), g, dim3(BA_WG), 0, s, a);
    else if (count32) hipLaunchKernelGGL((k_bucket_agg<false, true>), g, dim3(BA_WG), 0, s, a);
    else hipLaunchKernelGGL((k_bucket_agg<false, false>), g, dim3(BA_WG), 0, s, a);
}

void mrg_launch_table_clear(const TableArgs &t, bool indexer, hipStream_t s) {
    hipLaunchKernelGGL(k_table_clear, grid_for(t.cap), dim3(256), 0, s, t, indexer);
}
void mrg_launch_table_insert(const TableArgs &t, const uint64_t *k0, const uint64_t *k1, const uint32_t *cnt32,
                             const uint32_t *doc, uint64_t n, bool indexer, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_table_insert, grid_for(n), dim3(256), 0, s, t, k0, k1, cnt32, doc, n, indexer);
}
void mrg_launch_table_insert_x(const TableArgs &t, const XRec *x, uint64_t n, bool indexer, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_table_insert_x, grid_for(n), dim3(256), 0, s, t, x, n, indexer);
}
void mrg_launch_table_insert_l(const TableArgs &t, const LRec *x, uint64_t n, bool indexer, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_table_insert_l, grid_for(n), dim3(256), 0, s, t, x, n, indexer);
}
void mrg_launch_table_compact(const TableArgs &t, bool indexer, KeySet out, unsigned long long *counter,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_table_compact, grid_for(t.cap, TC_WG), dim3(TC_WG), 0, s, t, indexer, out, counter);
}
void mrg_launch_partition(KeySet ks, const uint8_t *heap, uint64_t n, uint32_t n_reduce, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_partition, grid_for(n), dim3(256), 0, s, ks, heap, n, n_reduce);
}
void mrg_launch_long_group(const uint64_t *fp_sorted, const uint32_t *idx_sorted, const uint32_t *doc,
                           const uint8_t *heap, const uint64_t *hoff, const uint32_t *flen, uint64_t n,
                           uint32_t *rep, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_long_group, grid_for(n), dim3(256), 0, s, fp_sorted, idx_sorted, doc, heap, hoff, flen, n,
                       rep);
}
void mrg_launch_long_emit(const uint32_t *rep, const uint64_t *cnt_in, const uint64_t *k0, const uint64_t *k1,
                          const uint32_t *flen, const uint64_t *hoff, const uint32_t *doc, uint64_t n,
                          unsigned long long *acc, KeySet out, unsigned long long *counter, bool indexer,
                          hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_long_count, grid_for(n), dim3(256), 0, s, rep, cnt_in, n, acc);
    hipLaunchKernelGGL(k_long_emit, grid_for(n), dim3(256), 0, s, rep, k0, k1, flen, hoff, doc, n,
                       (const unsigned long long *)acc, out, counter, indexer);
}
void mrg_launch_x_split_long(const XRec *x, uint64_t n, const uint64_t *seg_rec_end, const uint64_t *seg_heap_base,
                             uint32_t n_segs, LongItems li, unsigned long long *counter, bool indexer, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_x_split_long, grid_for(n), dim3(256), 0, s, x, n, seg_rec_end, seg_heap_base, n_segs, li,
                       counter, indexer);
}
void mrg_launch_l_split_long(const LRec *x, uint64_t n, const uint64_t *seg_rec_end, const uint64_t *seg_heap_base,
                             uint32_t n_segs, LongItems li, unsigned long long *counter, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_l_split_long, grid_for(n), dim3(256), 0, s, x, n, seg_rec_end, seg_heap_base, n_segs, li,
                       counter);
}
void mrg_launch_export_count(KeySet ks, uint64_t n, uint32_t n_owners, unsigned long long *rec_cnt,
                             unsigned long long *heap_cnt, bool indexer, uint64_t vmax, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_export_count, grid_for(n, EXP_WG), dim3(EXP_WG), 0, s, ks, n, n_owners, rec_cnt, heap_cnt,
                       indexer, vmax);
}
void mrg_launch_export_pack(KeySet ks, const uint8_t *heap, uint64_t n, uint32_t n_owners,
                            const uint64_t *rec_base, const uint64_t *heap_base, unsigned long long *rec_cur,
                            unsigned long long *heap_cur, XRec *out, uint8_t *out_heap, bool indexer, uint64_t vmax,
                            hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_export_pack, grid_for(n, EXP_WG), dim3(EXP_WG), 0, s, ks, heap, n, n_owners, rec_base,
                       heap_base, rec_cur, heap_cur, out, out_heap, indexer, vmax);
}
void mrg_launch_make_sortrec(KeySet ks, uint64_t n, const uint32_t *doc_rank, void *recs, hipStream_t s, bool carry) {
    if (!n) return;
    hipLaunchKernelGGL(k_make_sortrec, grid_for(n), dim3(256), 0, s, ks, n, doc_rank, (SortRec *)recs, carry ? 1 : 0);
}
void mrg_launch_wide_counts(const BucketArgs &a, uint64_t *cnt, uint64_t nseg, hipStream_t s) {
    hipLaunchKernelGGL(k_wide_counts, grid_for(nseg), dim3(256), 0, s, a, cnt);
}
void mrg_launch_wide_gather(const BucketArgs &a, const uint64_t *off, uint64_t nseg, uint32_t n_reduce, SortRec *out,
                            hipStream_t s) {
    hipLaunchKernelGGL(k_wide_gather, dim3((unsigned)nseg), dim3(256), 0, s, a, off, n_reduce, out);
}
void mrg_launch_wide_heads(const SortRec *r, uint64_t n, uint64_t *head, uint64_t *cv, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_wide_heads, grid_for(n), dim3(256), 0, s, r, n, head, cv);
}
void mrg_launch_wide_keys(const SortRec *r, uint64_t n, const uint64_t *head, const uint64_t *E, KeySet ks,
                          uint64_t *F, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_wide_keys, grid_for(n), dim3(256), 0, s, r, n, head, E, ks, F);
}
void mrg_launch_wide_cnt(const uint64_t *F, uint64_t runs, uint64_t n, const uint64_t *C, uint64_t ctot, KeySet ks,
                         hipStream_t s) {
    if (runs) hipLaunchKernelGGL(k_wide_cnt, grid_for(runs), dim3(256), 0, s, F, runs, n, C, ctot, ks);
}
void mrg_launch_fill_u32(uint32_t *p, uint32_t v, uint64_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_fill<uint32_t>, grid_for(n), dim3(256), 0, s, p, v, n);
}
void mrg_launch_fill_u64(uint64_t *p, uint64_t v, uint64_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_fill<uint64_t>, grid_for(n), dim3(256), 0, s, p, v, n);
}
void mrg_launch_iota_u32(uint32_t *p, uint64_t n, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_iota, grid_for(n), dim3(256), 0, s, p, n);
}
