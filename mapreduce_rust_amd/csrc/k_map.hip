// k_map.hip -- the map kernel: tokenize + local combine (MI355X / gfx950).
//
// Replaces wc::map (src/app/wc.rs:6-13) -- delete every codepoint outside \w ∪ \s, split on
// White_Space -- fused with the per-token part of write_key_value_to_file (src/mr/worker.rs:127-131).
// The partition index (worker.rs:129) is computed later, once per DISTINCT key (k_keys.hip), since
// SipHash(key) % R is a pure function of the key.  Also validates UTF-8 like read_to_string
// (worker.rs:75): the first invalid byte offset is reported and the job fails with MRG_EUTF8.
//
// Layout: documents back to back in one HBM buffer; each document is cut into 1 KiB
// tiles on a 16-byte-aligned grid.  A persistent grid of 512-thread workgroups (8 waves) walks the
// tiles, and every WAVE works on a tile of its own -- no workgroup barrier in the main loop: the
// wave's next tile (64 lanes x 16 B + halo) is in flight in registers while it processes the
// current one from its private LDS window.  The 8 waves share the workgroup's combine table.
//
// ASCII tiles (the common case; wave-uniform test) take the fast path:
//   1. every lane classifies one 16-byte segment through a 128-entry LDS LUT into an interleaved
//      32-bit mask (bit 2k = byte k is \w, bit 2k+1 = byte k is White_Space);
//   2. token starts = non-space bytes after a space: mask arithmetic, the previous byte's class
//      from the neighbour lane (shuffle); the wave compacts its starts into an LDS queue (prefix
//      sum) so that all 64 lanes then work on one token each;
//   3. per token: end = next space bit, key = the \w bytes -- contiguous unless a deleted byte sits
//      inside the token ("don't") -- read as 3 x 8 B from LDS and packed big-endian into (k0, k1);
//      > 31-byte raw tokens and tokens running past the halo take the exact per-codepoint walker.
// Non-ASCII tiles use the per-codepoint walker for every token (UTF-8 decode + class table).
// Keys of <= 16 bytes go to the workgroup's LDS hash table (exact: the packed key IS the identity)
// of 8-slot tagged groups; a miss is appended to one of 512 hash buckets in HBM, into the region
// this workgroup owns in that bucket (an LDS cursor per bucket: no HBM atomics).  Keys > 16 bytes
// become long-token records (start, raw length, doc) resolved by the collision-safe fingerprint
// sort (k_keys.hip).  At the end the LDS table is flushed, sorted by bucket, into the workgroup's
// flush region.
#include "mrg_device.h"
#include "mrg_internal.h"

namespace {

constexpr int WG = MRG_MAP_WG;
constexpr int NWAVE = WG / 64;
constexpr int SEG = MRG_MAP_SEG;
constexpr int TILE = MRG_MAP_TILE;
constexpr int HALO = MRG_MAP_HALO;
constexpr int BEHIND = MRG_MAP_BEHIND;
constexpr int NSEG = TILE / SEG + 1;                // classified segments: tile + first halo segment
constexpr int LDS_BYTES = BEHIND + TILE + HALO + 32;  // per wave (+32: 3 x 8 B key reads at the edge)
constexpr int NVEC_MAX = (BEHIND + TILE + HALO + 15) / 16;  // staged 16-byte vectors per tile
constexpr int QCAP = TILE / 2;                      // tokens per tile <= 512
// queue entry (u32): start (10 bits) | raw length n << 10 | key span first << 16 | L << 21 | kind << 27
constexpr uint32_t QK_PLAIN = 0;  // \w bytes contiguous: key = bytes [first, first + L) of the token
constexpr uint32_t QK_INNER = 1;  // deleted bytes inside the token ("don't")
constexpr uint32_t QK_SLOW = 2;   // longer than the 2-segment window or cut by the staged edge: walker
constexpr uint32_t QK_EMPTY = 3;  // no \w byte: not a token
constexpr uint64_t SBITS = 0xAAAAAAAAAAAAAAAAull;    // odd bits: White_Space flags
constexpr uint64_t WBITS = 0x5555555555555555ull;    // even bits: \w flags
static_assert(NVEC_MAX <= 128, "two prefetch vectors per lane");
static_assert(TILE == 64 * SEG, "one segment per lane");

// LDS-staged window: byte a lives at lds[a - wbase] when lo <= a < hi, else it is read from HBM.
struct Window {
    const uint8_t *lds;
    const uint8_t *g;
    uint64_t lo, hi, wbase;
    __device__ __forceinline__ uint32_t operator()(uint64_t a) const {
        return (a >= lo && a < hi) ? (uint32_t)lds[a - wbase] : (uint32_t)g[a];
    }
};

struct TileInfo {
    uint64_t At, t0, t1, doc_lo, doc_hi, wlo, whi;
    uint32_t docid, v0, v1;
};

// Tile c of the job.  A wave visits its tiles in increasing order, so the document index only moves
// forward from the previous tile's (usually not at all).
__device__ __forceinline__ TileInfo locate(const MapArgs &A, uint64_t c, uint32_t &d) {
    while (A.chunk_base[d + 1] <= c) ++d;  // chunk_base[d] <= c < chunk_base[d+1]
    const uint32_t lo_d = d;
    TileInfo t;
    t.doc_lo = A.doc_off[lo_d];
    t.doc_hi = A.doc_off[lo_d + 1];
    t.At = (t.doc_lo & ~15ull) + (c - A.chunk_base[lo_d]) * (uint64_t)TILE;  // aligned tile base
    t.t0 = max(t.At, t.doc_lo);
    t.t1 = min(t.At + (uint64_t)TILE, t.doc_hi);
    t.docid = A.doc_id ? A.doc_id[lo_d] : lo_d;
    const uint64_t wbase = t.At - (uint64_t)BEHIND;  // may wrap below 0: only differences are used
    t.wlo = max(t.doc_lo, t.At >= (uint64_t)BEHIND ? t.At - BEHIND : 0ull);
    t.whi = min(t.t1 + (uint64_t)HALO, t.doc_hi);
    t.v0 = (uint32_t)(((t.wlo & ~15ull) - wbase) >> 4);
    t.v1 = (uint32_t)((((t.whi + 15u) & ~15ull) - wbase) >> 4);
    return t;
}

__device__ __forceinline__ void report_error(unsigned long long *counters, uint64_t pos) {
    atomicMin(&counters[CNT_ERRPOS], (unsigned long long)pos);
}

__device__ __forceinline__ uint32_t key_hash(uint64_t k0, uint64_t k1, uint32_t d, uint32_t hash_bits) {
    uint32_t h = mrg_key_hash32(k0, k1, d);
    if (hash_bits && hash_bits < 32) h &= (1u << hash_bits) - 1u;
    return h;
}
__device__ __forceinline__ uint32_t bucket_of(uint32_t h) { return h >> (32 - MRG_NBUCKET_LOG2); }

// exact per-byte zero test: bit 8j+7 set iff byte j of x is 0
__device__ __forceinline__ uint64_t zero_bytes(uint64_t x) {
    return ~(((x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | x) & 0x8080808080808080ull;
}

// Workgroup LDS combine table: groups of 8 slots; a slot holds an 8-bit tag (0 =
// empty), the packed key (k0, k1[, doc]) and a count.  Probe = one 8-byte read of the group's tags,
// then the key of each tag-matching slot.  A new key claims an empty slot by CAS on its tag word and
// then writes the key; a concurrent lookup that reads the slot before the key is written sees a
// mismatch (an unwritten k0 is 0, which no key has) and goes on, so at worst one key occupies two
// slots -- harmless, the table only pre-sums and every slot is flushed and summed again exactly.
// A count is only ever added to a slot whose key equals the token's key.
template <int CAP, bool IDX>
struct LdsTable {
    static constexpr uint32_t NG = CAP / 8;
    unsigned long long *k0, *k1;
    unsigned int *cnt, *doc;
    unsigned long long *tag;  // [NG]: the 8 tags of group g in bytes of tag[g]

    __device__ __forceinline__ bool matches(uint32_t s, uint64_t a, uint64_t b, uint32_t d) const {
        // both key words are read before either is compared: one LDS round trip, not two
        const uint64_t x = (k0[s] ^ a) | (k1[s] ^ b);
        return x == 0 && (!IDX || doc[s] == d);
    }

    __device__ __forceinline__ bool insert(uint64_t a, uint64_t b, uint32_t d, uint32_t h) {
        const uint32_t g = h & (NG - 1);
        const uint64_t tg = ((h >> 16) & 0xFFu) | 1u;            // nonzero 8-bit tag
        uint64_t tags = tag[g];
        uint64_t cand = zero_bytes(tags ^ (tg * 0x0101010101010101ull));
        while (cand) {
            const uint32_t s = g * 8u + ((uint32_t)__builtin_ctzll(cand) >> 3);
            if (matches(s, a, b, d)) {
                atomicAdd(&cnt[s], 1u);
                return true;
            }
            cand &= cand - 1u;
        }
        uint64_t empty = zero_bytes(tags);
        while (empty) {
            const uint32_t j = (uint32_t)__builtin_ctzll(empty) >> 3;
            const uint64_t want = tags | (tg << (8u * j));
            const uint64_t old = atomicCAS(&tag[g], tags, want);
            if (old == tags) {  // slot j claimed
                const uint32_t s = g * 8u + j;
                k0[s] = a;
                k1[s] = b;
                if (IDX) doc[s] = d;
                atomicAdd(&cnt[s], 1u);
                return true;
            }
            // the group changed under us: a slot we had not checked may now hold the key
            const uint64_t newly = zero_bytes(tags) & ~zero_bytes(old);
            uint64_t nc = zero_bytes(old ^ (tg * 0x0101010101010101ull)) & newly;
            while (nc) {
                const uint32_t s = g * 8u + ((uint32_t)__builtin_ctzll(nc) >> 3);
                if (matches(s, a, b, d)) {
                    atomicAdd(&cnt[s], 1u);
                    return true;
                }
                nc &= nc - 1u;
            }
            tags = old;
            empty = zero_bytes(tags);
        }
        return false;  // group full of other keys: miss
    }
};

// Walk ONE token whose first codepoint starts at `a` (the codepoint before `a` is White_Space or the
// document start): decode codepoints until White_Space or the document end, keep \w bytes.
// Returns false on invalid UTF-8 (reported).  *end = first byte after the token.
template <class RD>
__device__ __noinline__ bool walk_token(const RD &rd, uint64_t a, uint64_t doc_hi, unsigned long long *counters,
                                        uint64_t &k0, uint64_t &k1, uint32_t &L, uint64_t &end) {
    k0 = 0;
    k1 = 0;
    L = 0;
    uint64_t p = a;
    while (p < doc_hi) {
        uint32_t cp, raw;
        const int l = mrg_utf8_decode(rd, p, doc_hi, &cp, &raw);
        if (!l) {
            report_error(counters, p);
            end = p;
            return false;
        }
        const uint32_t c = mrg_uclass(cp);
        if (c == MRG_CLS_S) break;
        if (c == MRG_CLS_W) {
            for (int b = 0; b < l; ++b) {
                mrg_key_append(k0, k1, L, (raw >> (8 * b)) & 0xFFu);
                ++L;
            }
        }
        p += (uint64_t)l;
    }
    end = p;
    return true;
}

// One round of token emission by a whole wave (all 64 lanes must call it): LDS-table insert of short
// keys; a miss is appended to its hash bucket's region of this workgroup (an LDS counter per
// bucket, no HBM atomics).  Long keys become long-token records.
template <int CAP, bool IDX>
__device__ __forceinline__ void emit_round(const MapArgs &A, LdsTable<CAP, IDX> &table, uint32_t *bcount,
                                           const uint32_t *bcap, const unsigned long long *bbase, bool have,
                                           uint64_t tk0, uint64_t tk1, uint32_t tlen, uint64_t tstart, uint32_t traw,
                                           uint32_t docid) {
    const bool is_long = have && tlen > 16u;
    bool tail = false;
    uint32_t h = 0;
    const uint32_t dkey = IDX ? docid : MRG_EMPTY_DOC;
    if (have && !is_long) {
        h = key_hash(tk0, tk1, dkey, A.hash_bits);
        tail = (A.ablate & 2u) ? true : !table.insert(tk0, tk1, dkey, h);
    }
    if (tail && !(A.ablate & 1u)) {
        const uint32_t b = bucket_of(h);
        const uint32_t slot = atomicAdd(&bcount[b], 1u);
        uint64_t *dst = nullptr;
        if (slot < bcap[b]) {
            dst = A.pool + (bbase[b] + slot) * (IDX ? 3u : 2u);
        } else {  // region full (rare): the bucket's shared overflow list
            const uint32_t j = atomicAdd(&A.onext[b], 1u);
            if (j < A.ocap) dst = A.ovf + ((uint64_t)b * A.ocap + j) * (IDX ? 3u : 2u);
            else atomicAdd(&A.counters[CNT_OVF], 1ull);
        }
        if (dst) {
            dst[0] = tk0;
            dst[1] = tk1;
            if (IDX) dst[2] = docid;
        }
    }
    const uint64_t li = mrg_wave_append(&A.counters[CNT_LONG], is_long);
    if (is_long && li < A.lcap) {
        A.lstart[li] = tstart;
        A.llen[li] = traw;
        A.ldoc[li] = docid;
    }
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int CAP, bool IDX>
__global__ __launch_bounds__(WG, (CAP >= 4096 || (IDX && CAP >= 2048)) ? 2 : 4) void k_map(const MapArgs *__restrict__ Ap) {
    // the arguments live in device memory (not the kernarg segment): fields are loaded where they
    // are used instead of being held in SGPRs for the whole kernel
    const MapArgs &A = *Ap;
    // per wave: staged window, segment masks, token queue (waves work on their own tiles)
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[NWAVE][LDS_BYTES];
    __shared__ uint32_t s_mask[NWAVE][NSEG];
    __shared__ uint32_t s_queue[NWAVE][QCAP];
    __shared__ uint8_t s_lut[128];
    // workgroup: combine table + tail-region cursors
    __shared__ __attribute__((aligned(16))) unsigned long long s_k0[CAP];
    __shared__ __attribute__((aligned(16))) unsigned long long s_k1[CAP];
    __shared__ unsigned int s_cnt[CAP];
    __shared__ __attribute__((aligned(16))) unsigned int s_doc[IDX ? CAP : 1];
    __shared__ unsigned long long s_tag[CAP / 8];
    __shared__ uint32_t s_bcount[MRG_NBUCKET];           // records appended to (bucket, this WG)
    __shared__ uint32_t s_bcap[MRG_NBUCKET];
    __shared__ unsigned long long s_bbase[MRG_NBUCKET];  // first pool record of (bucket, this WG)
    __shared__ uint32_t s_hist[MRG_NBUCKET + 1];
    static_assert(sizeof(s_queue) >= CAP * sizeof(uint16_t), "flush ranks reuse the queues");

    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    for (int i = tid; i < CAP; i += WG) {
        s_k0[i] = MRG_EMPTY_K0;
        s_k1[i] = MRG_EMPTY_K1;
        s_cnt[i] = 0;
        if (IDX) s_doc[i] = MRG_EMPTY_DOC;
    }
    for (int i = tid; i < CAP / 8; i += WG) s_tag[i] = 0;
    for (int b = tid; b < MRG_NBUCKET; b += WG) {
        s_bcount[b] = 0;
        const uint32_t cap = A.bcap[b];
        s_bcap[b] = cap;
        s_bbase[b] = A.rbase[b] + (uint64_t)blockIdx.x * cap;
    }
    if (tid < 128) s_lut[tid] = (uint8_t)(mrg_uclass((uint32_t)tid) == MRG_CLS_W ? 1u
                                          : (mrg_uclass((uint32_t)tid) == MRG_CLS_S ? 2u : 0u));
    LdsTable<CAP, IDX> table{s_k0, s_k1, s_cnt, s_doc, s_tag};
    uint32_t my_tokens = 0;
    uint8_t *tile = s_tile[wv];
    uint32_t *mask = s_mask[wv];
    uint32_t *queue = s_queue[wv];
    __syncthreads();

    // Staged window of a tile, as 16-byte vectors j relative to At - 16: j = 0 the byte block before
    // the tile, j = 1..64 the tile's segments 0..63, j = 65..68 the halo.  Lane l holds vector 1 + l
    // (its own segment: classified straight from registers) in p0; lanes 0..4 hold vectors 0 and
    // 65..68 in p1.  Only vectors inside [v0, v1) are loaded (they never leave the allocation).
    const uint64_t stride = (uint64_t)gridDim.x * NWAVE;
    uint64_t c = (uint64_t)blockIdx.x * NWAVE + wv;
    uint32_t dcur = 0;
    const uint32_t j0 = 1u + (uint32_t)lane;
    const uint32_t j1 = lane == 0 ? 0u : 64u + (uint32_t)lane;
    const bool has1 = lane < 5;
    TileInfo nx{};
    uint4 pf0 = {0, 0, 0, 0}, pf1 = {0, 0, 0, 0};
    auto prefetch = [&](const TileInfo &t) {
        const uint4 *src = reinterpret_cast<const uint4 *>(A.in + (t.At - (uint64_t)BEHIND));
        pf0 = uint4{0, 0, 0, 0};
        pf1 = uint4{0, 0, 0, 0};
        if (j0 >= t.v0 && j0 < t.v1) pf0 = src[j0];
        if (has1 && j1 >= t.v0 && j1 < t.v1) pf1 = src[j1];
    };
    if (c < A.n_chunks) {
        nx = locate(A, c, dcur);
        prefetch(nx);
    }

    for (; c < A.n_chunks; c += stride) {
        const TileInfo T = nx;
        const uint4 x0 = pf0, x1 = pf1;
        Window W;
        W.lds = tile;
        W.g = A.in;
        W.wbase = T.At - (uint64_t)BEHIND;
        W.lo = T.wlo;
        W.hi = T.whi;

        // this wave finished its previous tile (program order): the buffers are free
        const bool in0 = j0 >= T.v0 && j0 < T.v1, in1 = has1 && j1 >= T.v0 && j1 < T.v1;
        if (in0) reinterpret_cast<uint4 *>(tile)[j0] = x0;
        if (in1) reinterpret_cast<uint4 *>(tile)[j1] = x1;
        const bool nonascii = (((x0.x | x0.y | x0.z | x0.w) | (x1.x | x1.y | x1.z | x1.w)) & 0x80808080u) != 0u;
        const bool generic = __any(nonascii);
        // next tile's loads fly while this one is processed
        if (c + stride < A.n_chunks) {
            nx = locate(A, c + stride, dcur);
            prefetch(nx);
        }
        const uint64_t At = T.At, t0 = T.t0, t1 = T.t1, doc_lo = T.doc_lo, doc_hi = T.doc_hi;
        const uint32_t docid = T.docid;

        if (generic) {
            wave_sync_lds();
            // ================= generic path: per-lane codepoint walker =================
            const uint64_t sg0 = At + (uint64_t)lane * SEG;
            const uint64_t s0 = max(sg0, t0);
            const uint64_t s1 = min(sg0 + (uint64_t)SEG, t1);
            bool done = s0 >= s1;
            uint64_t p = s0;
            bool prevS = true;
            if (!done && s0 > doc_lo) {
                uint32_t j = 0;  // continuation bytes belong to a codepoint that starts before s0
                while (s0 + j < s1 && mrg_is_cont(W(s0 + j))) ++j;
                p = s0 + j;
                uint32_t k = 1;  // lead of the codepoint ending at p - 1 (at most 3 continuation bytes back)
                while (k <= 3 && p - k >= doc_lo && mrg_is_cont(W(p - k))) ++k;
                const uint64_t q = p - k;
                if (q < doc_lo || mrg_is_cont(W(q))) {
                    report_error(A.counters, s0);  // orphan continuation bytes
                    done = true;
                } else {
                    uint32_t cp, raw;
                    const int l = mrg_utf8_decode(W, q, doc_hi, &cp, &raw);
                    if (j > 0 && (l == 0 || q + (uint64_t)l != p)) {
                        report_error(A.counters, s0);
                        done = true;
                    }
                    prevS = (l > 0 && q + (uint64_t)l == p) ? (mrg_uclass(cp) == MRG_CLS_S) : false;
                }
                if (p >= s1) done = true;
            }
            for (;;) {
                bool have = false;
                uint64_t tk0 = 0, tk1 = 0, tstart = 0;
                uint32_t tlen = 0, traw = 0;
                while (!done) {
                    if (p >= s1) { done = true; break; }
                    uint32_t cp, raw;
                    const int l = mrg_utf8_decode(W, p, doc_hi, &cp, &raw);
                    if (!l) { report_error(A.counters, p); done = true; break; }
                    const uint32_t cl = mrg_uclass(cp);
                    if (cl == MRG_CLS_S) { prevS = true; p += (uint64_t)l; continue; }
                    if (!prevS) { p += (uint64_t)l; continue; }
                    uint64_t a0, a1, e;
                    uint32_t L;
                    if (!walk_token(W, p, doc_hi, A.counters, a0, a1, L, e)) { done = true; break; }
                    prevS = false;
                    const uint64_t start = p;
                    p = e;
                    if (L > 0) {
                        have = true;
                        tk0 = a0; tk1 = a1; tlen = L; tstart = start; traw = (uint32_t)(e - start);
                        break;
                    }
                }
                if (!__any(have)) break;
                my_tokens += have ? 1u : 0u;
                emit_round(A, table, s_bcount, s_bcap, s_bbase, have, tk0, tk1, tlen, tstart, traw, docid);
            }
            continue;
        }

        // ================= ASCII fast path =================
        // positions relative to At fit 32 bits: the tile is 1 KiB, the staged window ends at hi_rel
        const uint32_t hi_rel = (uint32_t)(W.hi - At);          // <= 1024 + HALO
        const bool cut = W.hi < doc_hi;                          // staged window ends inside the document
        const uint32_t t1_rel = (uint32_t)(t1 - At);
        const uint32_t lo_rel = doc_lo > At ? (uint32_t)(doc_lo - At) : 0u;
        // 1. classify: segment g covers [At + 16 g, +16); bytes outside [doc_lo, W.hi) count as space.
        auto classify = [&](const uint4 &x, uint32_t g) -> uint32_t {
            const uint32_t B = g * SEG;
            if (B >= hi_rel) return 0xAAAAAAAAu;
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t w = k == 0 ? x.x : (k == 1 ? x.y : (k == 2 ? x.z : x.w));
                m |= (uint32_t)s_lut[w & 0x7Fu] << (8 * k);
                m |= (uint32_t)s_lut[(w >> 8) & 0x7Fu] << (8 * k + 2);
                m |= (uint32_t)s_lut[(w >> 16) & 0x7Fu] << (8 * k + 4);
                m |= (uint32_t)s_lut[w >> 24] << (8 * k + 6);
            }
            const uint32_t lo_inv = lo_rel > B ? min(lo_rel - B, 16u) : 0u;
            const uint32_t hi_ok = min(hi_rel - B, 16u);
            const uint32_t vhi = hi_ok >= 16u ? 0xFFFFFFFFu : ((1u << (2u * hi_ok)) - 1u);
            const uint32_t vlo = lo_inv >= 16u ? 0xFFFFFFFFu : ((1u << (2u * lo_inv)) - 1u);
            const uint32_t valid = vhi & ~vlo;
            return (m & valid) | (0xAAAAAAAAu & ~valid);
        };
        const uint32_t m = classify(x0, (uint32_t)lane);
        uint32_t m64 = lane == 1 ? classify(x1, 64u) : 0u;   // the first halo segment is lane 1's p1
        m64 = __builtin_amdgcn_readlane(m64, 1);
        mask[lane] = m;
        if (lane == 0) mask[64] = m64;
        uint32_t mn = __shfl_down(m, 1);
        if (lane == 63) mn = m64;
        // 2. token starts of this lane's segment: the previous byte's class from lane l-1's mask (or
        //    the staged byte before the tile); each start becomes one queue entry that already knows
        //    its raw length, key span and kind, so a consumer lane reads the key bytes directly
        uint32_t prev = __shfl_up(m >> 31, 1);
        if (lane == 0) prev = At > doc_lo ? (s_lut[(x1.w >> 24) & 0x7Fu] >> 1) & 1u : 1u;
        const uint32_t IS = m & 0xAAAAAAAAu;
        uint32_t st = ~IS & ((IS << 2) | (prev << 1)) & 0xAAAAAAAAu;
        if ((uint32_t)lane * SEG >= t1_rel) st = 0;
        const uint32_t cnt = __popc(st);
        uint32_t incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o);
            if (lane >= o) incl += u;
        }
        uint32_t pos = incl - cnt;
        const uint64_t win = (uint64_t)m | ((uint64_t)mn << 32);
        while (st) {
            const uint32_t k = (uint32_t)__builtin_ctz(st) >> 1;
            st &= st - 1u;
            const uint32_t s = (uint32_t)lane * SEG + k;
            const uint64_t sr = (win & SBITS) >> (2u * k + 2u);
            uint32_t n = 0, first = 0, L = 0, kind = QK_SLOW;
            if (sr) {
                n = ((uint32_t)__builtin_ctzll(sr) >> 1) + 1u;  // raw length
                if (!(cut && s + n >= hi_rel)) {                // not ended by the staged edge
                    const uint64_t w = (win >> (2u * k)) & WBITS & ((1ull << (2u * n)) - 1u);
                    if (!w) {
                        kind = QK_EMPTY;                        // no \w byte: no token
                    } else {
                        first = (uint32_t)__builtin_ctzll(w) >> 1;
                        const uint32_t last = (63u - (uint32_t)__builtin_clzll(w)) >> 1;
                        L = last - first + 1u;
                        const uint64_t pat = (WBITS >> (64u - 2u * L)) << (2u * first);
                        kind = w == pat ? QK_PLAIN : QK_INNER;
                    }
                }
            }
            queue[pos++] = s | (n << 10) | (first << 16) | (L << 21) | (kind << 27);
        }
        const uint32_t total = (A.ablate & 4u) ? 0u : __shfl(incl, 63);
        my_tokens += (A.ablate & 4u) ? cnt : 0u;
        wave_sync_lds();

        // 3. tokens of the queue, one per lane per round (queue, masks and tile are read-only now)
        for (uint32_t base = 0; base < total; base += 64) {
            const uint32_t q = base + lane;
            bool have = false;
            uint64_t tk0 = 0, tk1 = 0;
            uint32_t tlen = 0, traw = 0, s = 0;
            if (q < total) {
                const uint32_t e = queue[q];
                s = e & 1023u;
                const uint32_t n = (e >> 10) & 63u, first = (e >> 16) & 31u, L = (e >> 21) & 63u, kind = e >> 27;
                if (kind == QK_PLAIN) {
                    have = true;
                    tlen = L;
                    traw = n;
                    if (L <= 16u) {
                        const uint32_t off = BEHIND + s + first;
                        const uint64_t *q64 = reinterpret_cast<const uint64_t *>(tile + (off & ~7u));
                        const uint64_t y0 = q64[0], y1 = q64[1], y2 = q64[2];
                        const uint32_t sh = (off & 7u) * 8u;
                        uint64_t lo = sh ? (y0 >> sh) | (y1 << (64u - sh)) : y0;
                        uint64_t hi = sh ? (y1 >> sh) | (y2 << (64u - sh)) : y1;
                        if (L < 8u) { lo &= (1ull << (8u * L)) - 1u; hi = 0; }
                        else if (L < 16u) hi &= (1ull << (8u * (L - 8u))) - 1u;
                        tk0 = __builtin_bswap64(lo);
                        tk1 = __builtin_bswap64(hi);
                    }
                } else if (kind == QK_INNER) {
                    // deleted (X) bytes inside an ASCII token ("don't"): keep the \w bytes
                    const uint32_t g = s >> 4, i = s & 15u;
                    const uint64_t wn = (uint64_t)mask[g] | ((uint64_t)mask[g + 1] << 32);
                    const uint64_t w = (wn >> (2u * i)) & WBITS & ((1ull << (2u * n)) - 1u);
                    uint64_t a0 = 0, a1 = 0;
                    uint32_t LL = 0;
                    for (uint32_t j = first; j < first + L; ++j) {
                        if ((w >> (2u * j)) & 1u) {
                            mrg_key_append(a0, a1, LL, tile[BEHIND + s + j]);
                            ++LL;
                        }
                    }
                    have = true;
                    tlen = LL;
                    traw = n;
                    tk0 = a0;
                    tk1 = a1;
                } else if (kind == QK_SLOW) {
                    uint64_t a0, a1, e2;
                    uint32_t L2;
                    if (walk_token(W, At + s, doc_hi, A.counters, a0, a1, L2, e2) && L2 > 0) {
                        have = true;
                        tk0 = a0; tk1 = a1; tlen = L2; traw = (uint32_t)(e2 - (At + s));
                    }
                }
            }
            my_tokens += have ? 1u : 0u;
            emit_round(A, table, s_bcount, s_bcap, s_bbase, have, tk0, tk1, tlen, At + s, traw, docid);
        }
    }

    // ---- flush the LDS table into this workgroup's region, sorted by bucket
    __syncthreads();
    uint16_t *s_rank = reinterpret_cast<uint16_t *>(&s_queue[0][0]);
    uint32_t *bcount = A.bcount + (uint64_t)blockIdx.x * MRG_NBUCKET;
    uint32_t my_tail = 0;
    for (int b = tid; b < MRG_NBUCKET; b += WG) {
        my_tail += s_bcount[b];
        bcount[b] = s_bcount[b];
    }
    for (int b = tid; b <= MRG_NBUCKET; b += WG) s_hist[b] = 0;
    __syncthreads();
    for (int i = tid; i < CAP; i += WG) {
        if (s_k0[i] == MRG_EMPTY_K0) continue;
        const uint32_t b = bucket_of(key_hash(s_k0[i], s_k1[i], IDX ? s_doc[i] : MRG_EMPTY_DOC, A.hash_bits));
        s_rank[i] = (uint16_t)atomicAdd(&s_hist[b], 1u);
    }
    __syncthreads();
    if (tid < 64) {  // exclusive scan of the bucket histogram by one wave
        uint32_t run = 0;
        for (int b0 = 0; b0 < MRG_NBUCKET; b0 += 64) {
            const uint32_t v = s_hist[b0 + lane];
            uint32_t inc = v;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = __shfl_up(inc, o);
                if (lane >= o) inc += u;
            }
            s_hist[b0 + lane] = run + inc - v;
            run += __shfl(inc, 63);
        }
        if (lane == 0) s_hist[MRG_NBUCKET] = run;
    }
    __syncthreads();
    uint32_t *foff = A.foff + (uint64_t)blockIdx.x * (MRG_NBUCKET + 1);
    for (int b = tid; b <= MRG_NBUCKET; b += WG) foff[b] = s_hist[b];
    const uint64_t reg = (uint64_t)blockIdx.x * CAP;
    for (int i = tid; i < CAP; i += WG) {
        if (s_k0[i] == MRG_EMPTY_K0) continue;
        const uint32_t d = IDX ? s_doc[i] : MRG_EMPTY_DOC;
        const uint32_t b = bucket_of(key_hash(s_k0[i], s_k1[i], d, A.hash_bits));
        const uint64_t pos2 = reg + s_hist[b] + s_rank[i];
        A.fk0[pos2] = s_k0[i];
        A.fk1[pos2] = s_k1[i];
        A.fcnt[pos2] = s_cnt[i];
        if (IDX) A.fdoc[pos2] = d;
    }
    uint32_t t = my_tokens, tl = my_tail;
    for (int off = 32; off > 0; off >>= 1) {
        t += __shfl_down(t, off);
        tl += __shfl_down(tl, off);
    }
    if (lane == 0) {
        atomicAdd(&A.counters[CNT_TOKENS], (unsigned long long)t);
        atomicAdd(&A.counters[CNT_REC], (unsigned long long)tl);
    }
}

// Long tokens: filter the raw token bytes (drop X codepoints), fingerprint (FNV-1a-64 of the key
// bytes; internal grouping only), packed prefix and key length.  Input was validated by k_map.
__global__ void k_long_prep(const uint8_t *in, const uint64_t *lstart, const uint32_t *llen, uint64_t n,
                            uint64_t *ok0, uint64_t *ok1, uint32_t *oflen, uint64_t *oflen64, uint64_t *ofp,
                            uint32_t hash_bits) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = lstart[i], e = a + llen[i];
    auto rd = [&](uint64_t x) -> uint32_t { return in[x]; };
    uint64_t k0 = 0, k1 = 0, h = 0xcbf29ce484222325ull;
    uint32_t L = 0;
    for (uint64_t p = a; p < e;) {
        uint32_t cp, raw;
        int l = mrg_utf8_decode(rd, p, e, &cp, &raw);
        if (!l) l = 1;  // cannot happen on validated input
        if (mrg_uclass(cp) == MRG_CLS_W) {
            for (int b = 0; b < l; ++b) {
                const uint32_t by = (raw >> (8 * b)) & 0xFFu;
                mrg_key_append(k0, k1, L, by);
                h = (h ^ by) * 0x100000001b3ull;
                ++L;
            }
        }
        p += (uint64_t)l;
    }
    if (hash_bits) h &= (1ull << hash_bits) - 1u;
    ok0[i] = k0; ok1[i] = k1; oflen[i] = L; oflen64[i] = L; ofp[i] = h;
}

// Copy the filtered key bytes of long token i to heap[dst_off[i] ..).
__global__ void k_long_gather(const uint8_t *in, const uint64_t *lstart, const uint32_t *llen, uint64_t n,
                              const uint64_t *dst_off, uint8_t *heap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = lstart[i], e = a + llen[i];
    auto rd = [&](uint64_t x) -> uint32_t { return in[x]; };
    uint8_t *dst = heap + dst_off[i];
    for (uint64_t p = a; p < e;) {
        uint32_t cp, raw;
        int l = mrg_utf8_decode(rd, p, e, &cp, &raw);
        if (!l) l = 1;
        if (mrg_uclass(cp) == MRG_CLS_W)
            for (int b = 0; b < l; ++b) *dst++ = (uint8_t)(raw >> (8 * b));
        p += (uint64_t)l;
    }
}

}  // namespace

template <int CAP, bool IDX>
static void launch_map_t(const MapArgs *a, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_map<CAP, IDX>), dim3(grid), dim3(WG), 0, s, a);
}

void mrg_launch_map(const MapArgs &h, MapArgs *a, int app, int grid, int lds_cap, hipStream_t s) {
    const bool idx = app == 1;
    (void)hipMemcpyAsync(a, &h, sizeof(MapArgs), hipMemcpyHostToDevice, s);
    if (lds_cap >= 4096) { if (idx) launch_map_t<4096, true>(a, grid, s); else launch_map_t<4096, false>(a, grid, s); }
    else if (lds_cap >= 2048) { if (idx) launch_map_t<2048, true>(a, grid, s); else launch_map_t<2048, false>(a, grid, s); }
    else { if (idx) launch_map_t<1024, true>(a, grid, s); else launch_map_t<1024, false>(a, grid, s); }
}

int mrg_map_cap(int lds_cap) { return lds_cap >= 4096 ? 4096 : (lds_cap >= 2048 ? 2048 : 1024); }

// tiles of a document [lo, hi): on the 16-byte grid starting at lo & ~15
uint64_t mrg_map_tiles(uint64_t lo, uint64_t hi) {
    if (hi <= lo) return 0;
    return (hi - (lo & ~15ull) + TILE - 1) / TILE;
}

int mrg_map_max_grid(int app, int lds_cap, int device) {
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
    int per = 1;
    const bool idx = app == 1;
    hipError_t e;
    if (lds_cap >= 4096) e = idx ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<4096, true>, WG, 0)
                                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<4096, false>, WG, 0);
    else if (lds_cap >= 2048) e = idx ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<2048, true>, WG, 0)
                                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<2048, false>, WG, 0);
    else e = idx ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<1024, true>, WG, 0)
                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<1024, false>, WG, 0);
    if (e != hipSuccess || per < 1) per = 1;
    return ncu * per;
}

void mrg_launch_long_prep(const uint8_t *base, const uint64_t *start, const uint32_t *rawlen, uint64_t n,
                          uint64_t *k0, uint64_t *k1, uint32_t *flen, uint64_t *flen64, uint64_t *fp,
                          uint32_t hash_bits, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_long_prep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, base, start, rawlen, n, k0,
                       k1, flen, flen64, fp, hash_bits);
}

void mrg_launch_long_gather(const uint8_t *base, const uint64_t *start, const uint32_t *rawlen, uint64_t n,
                            const uint64_t *dst_off, uint8_t *heap, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_long_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, base, start, rawlen, n,
                       dst_off, heap);
}
