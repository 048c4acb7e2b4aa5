// k_map.hip -- the map kernel: tokenize + local combine (MI355X / gfx950).
//
// Replaces wc::map (src/app/wc.rs:6-13) -- delete every codepoint outside \w ∪ \s, split on
// White_Space -- fused with the per-token part of write_key_value_to_file (src/mr/worker.rs:127-131).
// The partition index (worker.rs:129) is computed later, once per DISTINCT key (k_keys.hip), since
// SipHash(key) % R is a pure function of the key.  Also validates UTF-8 like read_to_string
// (worker.rs:75): the first invalid byte offset is reported and the job fails with MRG_EUTF8.
//
// Layout: documents back to back in one HBM buffer; each document is cut into 2 KiB
// blocks (two 1 KiB tiles) on a 16-byte-aligned grid.  One 16-wave workgroup per CU owns an equal
// share of the blocks; its waves take the next block from an LDS counter (no workgroup barrier in
// the main loop), with the next block's three 16-byte loads per lane in flight in registers (A/B
// register sets).  The 16 waves share the workgroup's LDS combine table.
//
// ASCII tiles (wave-uniform test) take the fast path, written for few instructions per byte:
//   1. lane l classifies its two 16-byte segments through a 128-entry byte LUT (32 dwords, one per
//      LDS bank) into W16 (\w) and S16 (White_Space) masks; the first halo segment by 16 lanes and
//      two ballots; token starts = non-space bytes after a space (the neighbour lane's last class by
//      DPP wave_shr); a DPP prefix sum gives every start a queue slot;
//   2. per tile each lane stores its 2-segment mask window (W and S of segments g, g+1) -- a consumer
//      lane reads ONE 8-byte word to find its token's raw length (first space), the \w span and
//      whether a deleted byte sits inside the token ("don't");
//   3. TWO tokens per lane per round (queue entries q and q + 64): 5 window dwords aligned to the
//      key's first byte (v_alignbyte) -> v_perm with a per-(length, 1-byte gap) selector from an LDS
//      table gives the big-endian packed key (k0, k1); further interior deletions are squeezed out
//      by 128-bit shifts; tokens that run past the 2-segment window or the staged halo are deferred
//      to the exact per-codepoint walker.
// Blocks with a non-ASCII byte take the same path with UTF-8-exact byte classes (each lane decodes
// the codepoints whose leads lie in its segments, in registers; when a lane holds two or more, the
// block's leads are first compacted one per lane through the wave's queue, see the block step); only blocks holding
// invalid UTF-8 are listed by the main loop and walked afterwards by all 16 waves with the exact
// per-codepoint walker, which reports the first bad byte.
// Keys of <= 16 bytes go to the workgroup's LDS hash table (exact: the packed key IS the identity):
// 4096 slots in 2-way sets, claimed only on a key's second sighting (a two-position Bloom
// doorkeeper).  A miss is appended to one of 256 hash buckets in HBM, into the region this workgroup
// owns in that bucket (one 64-bit LDS atomic on an absolute record cursor: no HBM atomics).  Keys > 16
// bytes become long-token records (start, raw length, doc) resolved by the collision-safe
// fingerprint sort (k_keys.hip).  At the end the LDS table is flushed, sorted by bucket, into the
// workgroup's flush region.
#include "mrg_device.h"
#include "mrg_internal.h"
#include "mrg_split.h"

namespace {

// Block rounds (r04, MRG_MAP_BR=1 in commit 5e363df, since removed): both tiles of a block tokenized
// by rounds of four tokens per lane with 12 waves per workgroup -- slower (157 VGPRs, 3 waves per
// SIMD).  Tiles are staged one at a time (a whole-block window needs the 16
// KiB that 16-byte table slots freed, and those slots cost ASCII text 3.5 %: section 11.1).
constexpr int NW = MRG_MAP_WAVES;
constexpr int WG = 64 * NW;
constexpr int SEG = MRG_MAP_SEG;
constexpr int TILE = MRG_MAP_TILE;
constexpr int HALO = MRG_MAP_HALO;
constexpr int BEHIND = MRG_MAP_BEHIND;
constexpr int NSUB = MRG_MAP_NSUB;               // 1 KiB tiles per block
constexpr int BLK = NSUB * TILE;                 // bytes per wave iteration
// staged window + slack for the 5-dword key reads (a key starts within 31 bytes of a token start)
constexpr int WIN = BEHIND + TILE + HALO + 48;
constexpr int QCAP = TILE / 2 + 16;  // token starts of a tile (a start needs a space before it)
constexpr int NMP = 64;         // mask pairs per wave (one per segment of the tile)
static_assert(TILE == 64 * SEG, "one segment per lane");
static_assert(WIN % 16 == 0, "16-byte window rows");
// Every tunable-sized LDS array against the largest index the code forms into it (the r05 fault in
// k_wleafw was a tunable outgrowing a fixed array: these fail the build instead).
//   mask pairs: mp[s >> 4] for a tile offset s < TILE, and mp[nseg - 1] with nseg <= TILE / SEG
static_assert(NMP == TILE / SEG, "one mask pair per segment of the tile");
//   window: the staged 16-byte vectors 0 .. 1 + TILE/16 + HALO/16 - 1 (the byte before, the tile,
//   the halo), and the key read's five dwords from BEHIND + s + first (s < TILE, first < 32)
static_assert(16 * (1 + TILE / 16 + HALO / 16) <= WIN, "staged vectors fit the window row");
static_assert(BEHIND + (TILE - 1) + 31 + 20 <= WIN, "the 5-dword key read stays in the window row");
static_assert(BEHIND == 16 && HALO % 16 == 0 && HALO >= 64, "one 16-byte vector behind, whole halo vectors");
//   queue: at most one token start per two bytes of the tile (a start follows a space), plus the
//   tile's first byte; reads are also clamped to QCAP - 1
static_assert(QCAP >= TILE / 2 + 1, "the token queue holds every start of a tile");
static_assert(BLK == 2 * TILE && NSUB == 2, "A/B register sets hold two tiles per lane (v0, v1)");

// ---------------------------------------------------------------- wave primitives (DPP, wave64)
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {  // lane l <- lane l+1 (lane 63 <- 0)
    return __builtin_amdgcn_update_dpp(0u, v, 0x130, 0xF, 0xF, false);  // wave_shl:1
}
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {  // lane l <- lane l-1 (lane 0 <- 0)
    return __builtin_amdgcn_update_dpp(0u, v, 0x138, 0xF, 0xF, false);  // wave_shr:1
}
// readlane / readfirstlane return int: wrap them so shifts and widening stay unsigned
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint32_t first_u32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
// a workgroup barrier for LDS only: the wave's outstanding global stores are not waited for (a
// __syncthreads() waits for them too -- at the end of the map that is every workgroup's last tail
// stores at once)
__device__ __forceinline__ void lds_only_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Global memory through address-space-1 pointers.  The kernel reads its pointers from a MapArgs in
// device memory, so without the cast every access would be a FLAT instruction -- and a pending FLAT
// op makes each LDS wait (lgkmcnt) also wait for every outstanding global load and store.
#define GAS __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ GAS T *gp(T *p) {
    return (GAS T *)p;
}
// Read-only job tables (document offsets, tile bases) through the constant address space: uniform
// loads become scalar loads (lgkmcnt), so the tile lookup never waits on the vector-memory counter
// -- which would also wait for the input prefetch issued just before it.
#define CAS __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ const CAS T *cp(const T *p) {
    return (const CAS T *)p;
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x3a __attribute__((ext_vector_type(3), aligned(4)));  // one 12-byte tail record
// byte-aligned LDS views (the key window read of the token rounds)
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));
template <class T>
__device__ __forceinline__ T g_add(T *p, T v) {
    return __hip_atomic_fetch_add(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 64-bit min/max as plain compares (HIP's overload set can resolve max(u64, u64) to the double
// version: a VALU f64 round trip per call)
__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }

struct TileInfo {
    uint64_t At, t0, t1, doc_lo, doc_hi, wlo, whi;
    uint32_t docid, v0, v1;
};

struct BlkInfo {
    uint64_t Ab, doc_lo, doc_hi;
    uint32_t docid, v0, v1;
};

// Block c of the job (BLK bytes on the document's 16-byte grid).  A wave visits its blocks in increasing
// order, so the document index only moves forward (usually not at all).  v0/v1: the loadable
// 16-byte vectors relative to Ab - 16 (the byte block before, the block, its 64-byte halo).
__device__ __forceinline__ BlkInfo locate_blk(const MapArgs &A, uint64_t c, uint32_t &d) {
    const CAS uint64_t *cb = cp(A.chunk_base), *doff = cp(A.doc_off);
    while (cb[d + 1] <= c) ++d;  // chunk_base[d] <= c < chunk_base[d+1]
    BlkInfo b;
    b.doc_lo = doff[d];
    b.doc_hi = doff[d + 1];
    b.Ab = (b.doc_lo & ~15ull) + (c - cb[d]) * (uint64_t)BLK;
    b.docid = A.doc_id ? cp(A.doc_id)[d] : d;
    const uint64_t vbase = b.Ab - (uint64_t)BEHIND;  // may wrap below 0: only differences are used
    const uint64_t wlo = umax64(b.doc_lo, b.Ab >= (uint64_t)BEHIND ? b.Ab - BEHIND : 0ull);
    const uint64_t whi = umin64(b.Ab + (uint64_t)(BLK + HALO), b.doc_hi);
    b.v0 = (uint32_t)(((wlo & ~15ull) - vbase) >> 4);
    b.v1 = (uint32_t)((((whi + 15u) & ~15ull) - vbase) >> 4);
    return b;
}

// Document of block c: the d with chunk_base[d] <= c < chunk_base[d + 1] (binary search; scalar).
__device__ __forceinline__ uint32_t find_doc(const MapArgs &A, uint64_t c) {
    const CAS uint64_t *cb = cp(A.chunk_base);
    uint32_t lo = 0, hi = A.n_docs;  // cb[lo] <= c < cb[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cb[mid] <= c) lo = mid;
        else hi = mid;
    }
    return lo;
}

// 1 KiB tile j of a block, with its staged window [At - 16, At + 1024 + 64) clipped to the document.
__device__ __forceinline__ TileInfo sub_tile(const BlkInfo &b, uint32_t j) {
    TileInfo t;
    t.At = b.Ab + (uint64_t)j * TILE;
    t.doc_lo = b.doc_lo;
    t.doc_hi = b.doc_hi;
    t.docid = b.docid;
    t.t0 = umax64(t.At, t.doc_lo);
    t.t1 = umin64(t.At + (uint64_t)TILE, t.doc_hi);
    const uint64_t wbase = t.At - (uint64_t)BEHIND;
    t.wlo = umax64(t.doc_lo, t.At >= (uint64_t)BEHIND ? t.At - BEHIND : 0ull);
    t.whi = umin64(t.t1 + (uint64_t)HALO, t.doc_hi);
    t.v0 = (uint32_t)(((t.wlo & ~15ull) - wbase) >> 4);
    t.v1 = (uint32_t)((((t.whi + 15u) & ~15ull) - wbase) >> 4);
    return t;
}

// timing variants only: an ablation compiled in as a constant (the product build: 0)
#ifndef MRG_MAP_ABL_CONST
#define MRG_MAP_ABL_CONST 0u
#endif
#ifndef MRG_MAP_CMPT  // compacted codepoint decode for blocks with a lane of 2+ leads (A/B switch)
#define MRG_MAP_CMPT 1
#endif
// per-wave dedup of a round's repeated keys (timing variant, MRG_MAP_DEDUP = leader rounds; 0 = off):
// see emit_fastN
#ifndef MRG_MAP_DEDUP
#define MRG_MAP_DEDUP 0
#endif

__device__ __forceinline__ uint32_t map_ablate(const MapArgs &A) {
#ifdef MRG_MAP_ABLATION
    return A.ablate;
#else
    (void)A;
    return MRG_MAP_ABL_CONST;
#endif
}

__device__ __forceinline__ void report_error(unsigned long long *counters, uint64_t pos) {
    __hip_atomic_fetch_min(gp(&counters[CNT_ERRPOS]), (unsigned long long)pos, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t key_hash(uint64_t k0, uint64_t k1, uint32_t d, uint32_t hash_bits) {
    uint32_t h = mrg_key_hash32(k0, k1, d);
    if (hash_bits && hash_bits < 32) h &= (1u << hash_bits) - 1u;
    return h;
}
__device__ __forceinline__ uint32_t bucket_of(uint32_t h) { return h >> (32 - MRG_NBUCKET_LOG2); }

// bit 8j+7 set where byte j of x is 0 -- exact when every byte is 0 or >= 0x80 (tag words), else it
// may also flag a 0x01 byte above a zero byte (candidate filter only: keys are always compared)
__device__ __forceinline__ uint64_t zero_bytes(uint64_t x) {
    return (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
}

struct alignas(16) KeyPair {
    uint64_t a, b;
};

// Workgroup LDS combine table: 2-way sets -- slots s and s + NS of set s = low
// hash bits (way-major: way 0 of the 2048 sets, then way 1, so a wave's 16-byte reads of one way
// spread over all 64 banks instead of half of them; A/B -0.5 % map).  A probe reads both keys at
// once (one LDS round trip: no tag step) and adds 1 to the
// matching slot's count.  A new key claims an empty way by a 64-bit CAS on k0 (EMPTY -> k0), then
// writes k1 (and doc) and adds its first count; slots only ever go EMPTY -> (k0, EMPTY) -> (k0, k1),
// so a slot read equal to the full key is that key's slot for good.  A reader that sees a half
// written slot, or a claimer that loses its CAS to the same k0, just misses -- harmless: misses go
// to the tail and every slot is flushed and summed exactly; at worst a key occupies both ways.
// (Measured by simulation at C3: 8-way tag groups 69.2 % hits, 2-way sets 68.1 %.)
//
// Admission (doorkeeper): a key may claim an empty way only on its second sighting in this
// workgroup -- the first sets its two bits in a 128 Kibit LDS Bloom filter (positions from the hash
// bits above the set index and from a remix of the hash; 32 Kibit for the indexer) and goes to the
// tail.  The table fills once and keeps its keys, so without the filter it
// fills with whatever the first few thousand tokens hold, singletons included; with it, mostly with
// repeated (frequent) keys.  Exactness is untouched: a token either adds to its key's slot or is
// appended to the tail, and both are summed.
#ifndef MRG_MAP_DOOR
#define MRG_MAP_DOOR 1
#endif
#ifndef MRG_MAP_DOOR_WORDS
#define MRG_MAP_DOOR_WORDS 4096
#endif
#ifndef MRG_MAP_DOOR_LEVELS
#define MRG_MAP_DOOR_LEVELS 1
#endif
static_assert(MRG_MAP_DOOR_WORDS >= 32 && (MRG_MAP_DOOR_WORDS & (MRG_MAP_DOOR_WORDS - 1)) == 0,
              "doorkeeper bit index is masked with DW * 32 - 1");
template <int CAP, bool IDX>
struct LdsTable {
    static constexpr uint32_t NS = CAP / 2;
    // the indexer's table has a doc word per slot: its bitmap stays at 32 Kibit to fit the LDS
    static constexpr uint32_t DW = (IDX && MRG_MAP_DOOR_WORDS > 1024) ? 1024u : (uint32_t)MRG_MAP_DOOR_WORDS;
    KeyPair *key;
    unsigned int *cnt, *doc;
    unsigned int *door;
    unsigned int *fill;  // slots claimed so far (never decreases: a claimed slot keeps its key)

    // seen before in this workgroup?  (records this sighting; collisions only admit early).  With
    // two levels, entries are 2-bit: admitted from the third sighting on.
    __device__ __forceinline__ bool admitted(uint32_t h) {
        if (!MRG_MAP_DOOR) return true;
        if (MRG_MAP_DOOR_LEVELS == 1) {
            // a two-position Bloom filter: hash bits 11.. and a multiplicative remix of the hash
            // (fewer false "seen before" while the table fills: simulated on the C3 stream, hits
            // 72.2 -> 72.9 %); both atomics in flight together, and only on the claim path
            const uint32_t di = (h >> 11) & (DW * 32u - 1u);
            const uint32_t dj = ((h * 0x9E3779B1u) >> 15) & (DW * 32u - 1u);
            const uint32_t bi = 1u << (di & 31u), bj = 1u << (dj & 31u);
            const uint32_t oi = atomicOr(&door[di >> 5], bi), oj = atomicOr(&door[dj >> 5], bj);
            return (oi & bi) != 0u && (oj & bj) != 0u;
        }
        const uint32_t di = (h >> 11) & (DW * 16u - 1u);
        const uint32_t lo = 1u << (2u * (di & 15u)), hi = lo << 1;
        unsigned int *w = &door[di >> 4];
        if (!(atomicOr(w, lo) & lo)) return false;
        return (atomicOr(w, hi) & hi) != 0u;
    }

    __device__ __forceinline__ bool matches(uint32_t s, uint64_t a, uint64_t b, uint32_t d) const {
        const KeyPair k = key[s];  // one 16-byte LDS read
        return ((k.a ^ a) | (k.b ^ b)) == 0 && (!IDX || doc[s] == d);
    }

    // claim an empty way of set s0 (ways seen empty: e0, e1); true if the key got a slot and its count
    __device__ __forceinline__ bool claim(uint32_t s0, bool e0, bool e1, uint64_t a, uint64_t b, uint32_t d,
                                          uint32_t h, uint32_t add = 1u) {
        if (!admitted(h)) return false;
        for (uint32_t w = 0; w < 2; ++w) {
            if (!(w ? e1 : e0)) continue;
            const uint32_t s = s0 + w * NS;  // way w of set s0: way-major layout
            const unsigned long long old = atomicCAS(&key[s].a, (unsigned long long)MRG_EMPTY_K0, (unsigned long long)a);
            if (old == MRG_EMPTY_K0) {
                key[s].b = b;
                if (IDX) doc[s] = d;
                atomicAdd(&cnt[s], add);
                atomicAdd(fill, 1u);
                return true;
            }
            if (old == a) return false;  // being claimed by the same k0: miss (safe)
        }
        return false;
    }

    // one probe per lane (slow path: one token per lane)
    __device__ __forceinline__ bool insert_wave(bool act, uint64_t a, uint64_t b, uint32_t d, uint32_t h,
                                                uint32_t abl = 0) {
        const uint32_t s0 = act ? (h & (NS - 1)) : 0u;
        const KeyPair k0 = key[s0], k1 = key[s0 + NS];
        const bool m0 = act & (((k0.a ^ a) | (k0.b ^ b)) == 0) & (!IDX || doc[s0] == d);
        const bool m1 = act & !m0 & (((k1.a ^ a) | (k1.b ^ b)) == 0) & (!IDX || doc[s0 + NS] == d);
        bool hit = m0 | m1;
        if (hit && !(abl & 16u)) atomicAdd(&cnt[m0 ? s0 : s0 + NS], 1u);
        const bool e0 = k0.a == MRG_EMPTY_K0, e1 = k1.a == MRG_EMPTY_K0;
        const bool need = act && !hit && (e0 || e1);
        if (__any(need)) {
            if (need) hit = claim(s0, e0, e1, a, b, d, h);
        }
        return hit;
    }
};

// Walk ONE token whose first codepoint starts at `a` (the codepoint before `a` is White_Space or the
// document start): decode codepoints until White_Space or the document end, keep \w bytes.
// Returns false on invalid UTF-8 (reported).  *end = first byte after the token.
template <class RD>
__device__ __forceinline__ bool walk_token(const RD &rd, uint64_t a, uint64_t doc_hi, unsigned long long *counters,
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

// Tail regions of this workgroup, one per hash bucket b: cur[b] = the pool record index of the next
// append (starts at the region's first record), end[b] = one past the region's last record.  An
// append is ONE 64-bit LDS atomic that returns the record index itself, and the end is read beside
// it (it does not depend on the atomic), so a tail token costs one LDS round trip before its store.
struct TailRegions {
    unsigned long long *cur;
    const unsigned long long *end;
    unsigned long long *cur16;  // wc keys of 13..16 bytes: their own regions of 16-byte records
    const unsigned long long *end16;
    unsigned int *lcnt;         // long-token records of this workgroup so far (its region's cursor)
    // wide map: cursors of this workgroup's L1-bucket regions and the splitters (LDS)
    unsigned int *wcur;
    const uint64_t *wspl;
    const uint8_t *wix;
};

// Wide map: the L1 bucket of a short key (partition = SipHash-1-3 % R, worker.rs:111-115, 129; then
// the number of the partition's splitters <= key, through the LDS index when there is one)
__device__ __forceinline__ uint32_t wide_bucket(const MapArgs &A, const TailRegions &R, uint64_t k0, uint64_t k1) {
    const uint32_t r = part_of(k0, k1, A.wR);
    const uint32_t m = A.wB1r - 1u;
    if (m == 0u) return r;
    const uint64_t *sp = R.wspl + 2ull * r * m;
    uint32_t q;
    if (R.wix) {
        const uint8_t *ixr = R.wix + r * MRG_WIDE_IX1;
        const SplitIndex<8, uint8_t> li{sp, ixr, m, ixr[257]};
        q = li.upper(k0, k1);
    } else {
        uint32_t lo = 0, hi = m;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (key_lt(k0, k1, sp[2 * mid], sp[2 * mid + 1])) hi = mid;
            else lo = mid + 1;
        }
        q = lo;
    }
    return r * A.wB1r + q;
}

// Wide map: append short key (k0, k1) to its L1 bucket's region of this workgroup (an LDS cursor per
// bucket; the count goes on past the region's capacity so the host can size a rerun)
__device__ __forceinline__ void wide_store(const MapArgs &A, const TailRegions &R, bool act, uint64_t k0, uint64_t k1) {
    if (!act) return;
    const uint32_t b = wide_bucket(A, R, k0, k1);
    if (A.w12 && (uint32_t)k1 != 0u) {  // 12-byte regions: a key of 13..16 bytes to the bucket's list
        const uint32_t j = atomicAdd(&A.wl16n[b], 1u);
        if (j < A.wl16cap) *reinterpret_cast<GAS u64x2 *>(gp(A.wl16) + 2ull * ((uint64_t)b * A.wl16cap + j)) = u64x2{k0, k1};
        else g_add(&A.counters[CNT_W16], 1ull);
        return;
    }
    const uint32_t pos = atomicAdd(&R.wcur[b], 1u);
    if ((MRG_MAP_ABL_CONST & 4096u) && pos != 0xFFFFFFFFu) return;   // timing variant only: no record store
    if (pos < A.wcap) {
        const uint64_t i = ((uint64_t)b * gridDim.x + blockIdx.x) * A.wcap + pos;
#if MRG_MAP_ABL_CONST & 8192u   // timing variant: non-temporal record stores
        if (A.w12)
            __builtin_nontemporal_store(u32x3a{(uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)(k1 >> 32)},
                                        reinterpret_cast<GAS u32x3a *>(reinterpret_cast<GAS uint8_t *>(gp(A.wrec)) + 12u * i));
        else
            __builtin_nontemporal_store(u64x2{k0, k1}, reinterpret_cast<GAS u64x2 *>(gp(A.wrec) + 2u * i));
#else
        if (A.w12)
            *reinterpret_cast<GAS u32x3a *>(reinterpret_cast<GAS uint8_t *>(gp(A.wrec)) + 12u * i) =
                u32x3a{(uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)(k1 >> 32)};
        else
            *reinterpret_cast<GAS u64x2 *>(gp(A.wrec) + 2u * i) = u64x2{k0, k1};
#endif
    }
}

// wc tail record i: keys of <= 12 bytes as 12 bytes {k0, high word of k1} in pool, longer ones as
// {k0, k1} in pool16; the indexer's {k0, k1, doc} (24 B) in pool
template <bool IDX>
__device__ __forceinline__ void store_tail(GAS uint64_t *pool, GAS uint64_t *pool16, bool w16, uint64_t i, uint64_t k0,
                                           uint64_t k1, uint32_t doc) {
    if (IDX) {
        GAS uint64_t *dst = pool + i * 3u;
        dst[0] = k0;
        dst[1] = k1;
        dst[2] = doc;
    } else if (w16) {
        *reinterpret_cast<GAS u64x2 *>(pool16 + 2u * i) = u64x2{k0, k1};
    } else {
        *reinterpret_cast<GAS u32x3a *>(reinterpret_cast<GAS uint8_t *>(pool) + 12u * i) =
            u32x3a{(uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)(k1 >> 32)};
    }
}

// N tokens per lane through the LDS table in one instruction stream: the set reads, count adds and
// tail-cursor adds of all N are issued back to back, so every LDS round trip is paid once for N
// independent chains.  Same semantics as emit() applied to token 0, then 1, ...
template <int N, int CAP, bool IDX>
__device__ __forceinline__ void emit_fastN(const MapArgs &A, uint32_t abl, uint32_t hbits, LdsTable<CAP, IDX> &T,
                                           TailRegions R, GAS uint64_t *pool, GAS uint64_t *pool16,
                                           const bool (&has)[N], const uint64_t (&k0)[N], const uint64_t (&k1)[N],
                                           uint32_t docid, bool may_claim) {
    constexpr uint32_t NS = LdsTable<CAP, IDX>::NS;
    const uint32_t dkey = IDX ? docid : MRG_EMPTY_DOC;
    uint32_t h[N], s[N], b[N];
    bool act[N], w16[N], hit[N], m0[N];
    KeyPair kw0[N], kw1[N];
    uint64_t end[N];
#pragma unroll
    for (int t = 0; t < N; ++t) {
        h[t] = key_hash(k0[t], k1[t], dkey, hbits);
        act[t] = has[t] && !(abl & 2u);
    }
#if MRG_MAP_DEDUP
    // Per-wave dedup (timing variant): MRG_MAP_DEDUP leader rounds over the round's N x 64 tokens.  A
    // leader is the first token still pending; every token with the leader's key joins its group,
    // skips the probe and the count add, and the leader adds the group's size.  When the leader
    // misses the table, the members go to the tail with it (one record each, as without dedup).
    uint32_t gadd[N], grp[N];
    bool pend[N];
#pragma unroll
    for (int t = 0; t < N; ++t) {
        gadd[t] = 1u;
        grp[t] = 0xFFu;
        pend[t] = act[t] && !IDX;
    }
    uint32_t gl_lane[MRG_MAP_DEDUP], gl_tok[MRG_MAP_DEDUP];
#pragma unroll
    for (int g = 0; g < MRG_MAP_DEDUP; ++g) {
        gl_tok[g] = 0xFFu;
        gl_lane[g] = 0;
        uint64_t pm[N];
#pragma unroll
        for (int t = 0; t < N; ++t) pm[t] = __ballot(pend[t]);
        int tl0 = -1;
#pragma unroll
        for (int t = N - 1; t >= 0; --t)
            if (pm[t]) tl0 = t;
        if (tl0 < 0) break;
        uint64_t la = 0, lb = 0;
        uint32_t src = 0;
#pragma unroll
        for (int t = 0; t < N; ++t)
            if (t == tl0) {
                src = (uint32_t)__builtin_ctzll(pm[t]);
                la = __builtin_amdgcn_readlane(k0[t] & 0xFFFFFFFFull, src) |
                     ((uint64_t)__builtin_amdgcn_readlane(k0[t] >> 32, src) << 32);
                lb = __builtin_amdgcn_readlane(k1[t] & 0xFFFFFFFFull, src) |
                     ((uint64_t)__builtin_amdgcn_readlane(k1[t] >> 32, src) << 32);
            }
        uint32_t gs = 0;
        bool eq[N];
#pragma unroll
        for (int t = 0; t < N; ++t) {
            eq[t] = pend[t] && k0[t] == la && k1[t] == lb;
            gs += (uint32_t)__popcll(__ballot(eq[t]));
        }
        const uint32_t me = __lane_id();
#pragma unroll
        for (int t = 0; t < N; ++t) {
            if (!eq[t]) continue;
            pend[t] = false;
            if (t == tl0 && me == src) {
                gadd[t] = gs;
            } else {
                grp[t] = (uint32_t)g;
                act[t] = false;   // a member: no probe, no count
            }
        }
        gl_tok[g] = (uint32_t)tl0;
        gl_lane[g] = src;
    }
#endif
#pragma unroll
    for (int t = 0; t < N; ++t) {
        s[t] = act[t] ? (h[t] & (NS - 1)) : 0u;
        b[t] = bucket_of(h[t]);
        w16[t] = !IDX && (uint32_t)k1[t] != 0u;  // wc keys of 13..16 bytes: the 16-byte regions
    }
    // both ways of every set: 2N 16-byte reads in flight together, with the region ends
#pragma unroll
    for (int t = 0; t < N; ++t) {
        kw0[t] = T.key[s[t]];
        kw1[t] = T.key[s[t] + NS];
        end[t] = (w16[t] ? R.end16 : R.end)[b[t]];
    }
#pragma unroll
    for (int t = 0; t < N; ++t) {
        m0[t] = act[t] & (((kw0[t].a ^ k0[t]) | (kw0[t].b ^ k1[t])) == 0) & (!IDX || T.doc[s[t]] == dkey);
        const bool m1 = act[t] & !m0[t] & (((kw1[t].a ^ k0[t]) | (kw1[t].b ^ k1[t])) == 0) &
                        (!IDX || T.doc[s[t] + NS] == dkey);
        hit[t] = m0[t] | m1;
    }
    if (!(abl & 16u)) {
#pragma unroll
        for (int t = 0; t < N; ++t)
#if MRG_MAP_DEDUP
            if (hit[t]) atomicAdd(&T.cnt[m0[t] ? s[t] : s[t] + NS], gadd[t]);
#else
            if (hit[t]) atomicAdd(&T.cnt[m0[t] ? s[t] : s[t] + NS], 1u);
#endif
    }
    // empty ways exist only until the table has filled (wave-uniform: a stale count only means
    // an unneeded test)
    if (may_claim) {
        bool e0[N], e1[N], need[N], any = false;
#pragma unroll
        for (int t = 0; t < N; ++t) {
            e0[t] = kw0[t].a == MRG_EMPTY_K0;
            e1[t] = kw1[t].a == MRG_EMPTY_K0;
            need[t] = act[t] && !hit[t] && (e0[t] || e1[t]);
            any = any || need[t];
        }
        if (__any(any)) {
#pragma unroll
            for (int t = 0; t < N; ++t)
#if MRG_MAP_DEDUP
                if (need[t]) hit[t] = T.claim(s[t], e0[t], e1[t], k0[t], k1[t], dkey, h[t], gadd[t]);
#else
                if (need[t]) hit[t] = T.claim(s[t], e0[t], e1[t], k0[t], k1[t], dkey, h[t]);
#endif
        }
    }
#if MRG_MAP_DEDUP
    // members take their leader's outcome (a leader that missed: every member to the tail)
#pragma unroll
    for (int g = 0; g < MRG_MAP_DEDUP; ++g) {
        if (gl_tok[g] == 0xFFu) break;
        uint32_t lh = 0;
#pragma unroll
        for (int t = 0; t < N; ++t)
            if ((uint32_t)t == gl_tok[g]) lh = __builtin_amdgcn_readlane(hit[t] ? 1u : 0u, gl_lane[g]);
#pragma unroll
        for (int t = 0; t < N; ++t)
            if (grp[t] == (uint32_t)g) hit[t] = lh != 0u;
    }
#endif
    bool tl[N], anyt = false;
#pragma unroll
    for (int t = 0; t < N; ++t) {
        tl[t] = has[t] && !hit[t] && !(abl & 1u);
        anyt = anyt || tl[t];
    }
    // every token's append in one LDS round trip (a lane adds 0 for a token that hit)
    uint64_t idx[N];
    if (anyt) {
#pragma unroll
        for (int t = 0; t < N; ++t) idx[t] = atomicAdd(&(w16[t] ? R.cur16 : R.cur)[b[t]], tl[t] ? 1ull : 0ull);
    } else {
#pragma unroll
        for (int t = 0; t < N; ++t) idx[t] = 0;
    }
    bool anyo = false, ovf[N];
#pragma unroll
    for (int t = 0; t < N; ++t) {
        const bool ok = tl[t] && idx[t] < end[t];
        if (ok) store_tail<IDX>(pool, pool16, w16[t], idx[t], k0[t], k1[t], docid);
        ovf[t] = tl[t] && !ok;
        anyo = anyo || ovf[t];
    }
    if (__any(anyo)) {  // region full (rare): the bucket's shared overflow list
#pragma unroll
        for (int t = 0; t < N; ++t) {
            if (!ovf[t]) continue;
            const uint32_t j = g_add(&A.onext[b[t]], 1u);
            if (j < A.ocap) {
                GAS uint64_t *dst = gp(A.ovf) + ((uint64_t)b[t] * A.ocap + j) * (IDX ? 3u : 2u);
                dst[0] = k0[t];
                dst[1] = k1[t];
                if (IDX) dst[2] = docid;
            } else {
                g_add(&A.counters[CNT_OVF], 1ull);
            }
        }
    }
}

// One round of token emission by a whole wave (all 64 lanes call it): LDS-table insert of short
// keys; a miss is appended to its hash bucket's region of this workgroup (an LDS counter per
// bucket, no HBM atomics).  Long keys become long-token records.
template <int CAP, bool IDX, bool WIDE>
__device__ __forceinline__ void emit(const MapArgs &A, LdsTable<CAP, IDX> &table, TailRegions R, bool have,
                                     uint64_t tk0, uint64_t tk1, uint32_t tlen, uint64_t tstart, uint32_t traw,
                                     uint32_t docid) {
    const bool is_long = have && tlen > 16u;
    if constexpr (WIDE) {
        wide_store(A, R, have && !is_long, tk0, tk1);
    } else {
    bool tail = false;
    uint32_t h = 0;
    const uint32_t dkey = IDX ? docid : MRG_EMPTY_DOC;
    if (have && !is_long) {
        h = key_hash(tk0, tk1, dkey, A.hash_bits);
    }
    {
        const bool act = have && !is_long && !(map_ablate(A) & 2u);
        tail = (have && !is_long) && !table.insert_wave(act, tk0, tk1, dkey, h);
    }
    if (tail && !(map_ablate(A) & 1u)) {
        const uint32_t b = bucket_of(h);
        const bool w16 = !IDX && (uint32_t)tk1 != 0u;
        const uint64_t end = (w16 ? R.end16 : R.end)[b];
        const uint64_t idx = atomicAdd(&(w16 ? R.cur16 : R.cur)[b], 1ull);
        if (idx < end) {
            store_tail<IDX>(gp(A.pool), gp(A.pool16), w16, idx, tk0, tk1, docid);
        } else {  // region full (rare): the bucket's shared overflow list (16-byte records, any key)
            const uint32_t j = g_add(&A.onext[b], 1u);
            if (j < A.ocap) {
                GAS uint64_t *dst = gp(A.ovf) + ((uint64_t)b * A.ocap + j) * (IDX ? 3u : 2u);
                dst[0] = tk0;
                dst[1] = tk1;
                if (IDX) dst[2] = docid;
            } else {
                g_add(&A.counters[CNT_OVF], 1ull);
            }
        }
    }
    }
    // long tokens: the workgroup's own region through an LDS cursor (one LDS atomic per wave).  Until
    // r04 every such wave took its slots from ONE device-wide counter: a returning atomic on a single
    // address serialises chip-wide (~90 per microsecond), which bounded k_map on Gutenberg-like text,
    // where em-dash-joined words make ~1.2 M long tokens per 10 GiB, at ~14 ms.
    if (__any(is_long)) {
        const uint64_t mask = __ballot(is_long);
        const int leader = __ffsll((long long)mask) - 1;
        uint32_t base = 0;
        if ((int)__lane_id() == leader) base = atomicAdd(R.lcnt, (unsigned int)__popcll(mask));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
        const uint32_t k = base + (uint32_t)__popcll(mask & mrg_lanemask_lt());
        if (is_long) {
            uint64_t li = ~0ull;
            if (k < A.lper) {
                li = (uint64_t)blockIdx.x * A.lper + k;
            } else {  // region full (rare): the shared list
                const uint64_t j = g_add(&A.counters[CNT_LONGX], 1ull);
                if (j < A.lovf) li = (uint64_t)gridDim.x * A.lper + j;
            }
            if (li != ~0ull) {
                gp(A.lstart)[li] = tstart;
                gp(A.llen)[li] = traw;
                gp(A.ldoc)[li] = docid;
            }
        }
    }
}

// A tile with a non-ASCII byte: every lane walks the codepoints of its own 16-byte segment (UTF-8
// decode + two-level class table), one token per lane per emission round.  Called after the main
// loop (the main loop only records which tiles need it), so its registers never add to the hot
// loop's.
template <int CAP, bool IDX, bool WIDE>
__device__ __forceinline__ uint32_t generic_tile(const MapArgs &A, LdsTable<CAP, IDX> table, TailRegions R,
                                              const uint8_t *win, uint64_t At, uint64_t t0, uint64_t t1,
                                              uint64_t doc_lo, uint64_t doc_hi, uint64_t wlo, uint64_t whi,
                                              uint32_t docid) {
    const int lane = (int)__lane_id();
    const uint64_t wbase = At - (uint64_t)BEHIND;
    auto rd = [&](uint64_t a) -> uint32_t {
        if (a >= wlo && a < whi) return (uint32_t)win[a - wbase];
        return (uint32_t)gp(A.in)[a];
    };
    uint32_t my_tokens = 0;
        // ================= generic path: per-lane codepoint walker =================
        const uint64_t sg0 = At + (uint64_t)lane * SEG;
        const uint64_t s0 = umax64(sg0, t0);
        const uint64_t s1 = umin64(sg0 + (uint64_t)SEG, t1);
        bool done = s0 >= s1;
        uint64_t p = s0;
        bool prevS = true;
        if (!done && s0 > doc_lo) {
            uint32_t j = 0;  // continuation bytes belong to a codepoint that starts before s0
            while (s0 + j < s1 && mrg_is_cont(rd(s0 + j))) ++j;
            p = s0 + j;
            uint32_t k = 1;  // lead of the codepoint ending at p - 1 (at most 3 continuation bytes back)
            while (k <= 3 && p - k >= doc_lo && mrg_is_cont(rd(p - k))) ++k;
            const uint64_t q = p - k;
            if (q < doc_lo || mrg_is_cont(rd(q))) {
                report_error(A.counters, s0);  // orphan continuation bytes
                done = true;
            } else {
                uint32_t cp, raw;
                const int l = mrg_utf8_decode(rd, q, doc_hi, &cp, &raw);
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
                const int l = mrg_utf8_decode(rd, p, doc_hi, &cp, &raw);
                if (!l) { report_error(A.counters, p); done = true; break; }
                const uint32_t cl = mrg_uclass(cp);
                if (cl == MRG_CLS_S) { prevS = true; p += (uint64_t)l; continue; }
                if (!prevS) { p += (uint64_t)l; continue; }
                uint64_t a0w, a1w, e;
                uint32_t L;
                if (!walk_token(rd, p, doc_hi, A.counters, a0w, a1w, L, e)) { done = true; break; }
                prevS = false;
                const uint64_t start = p;
                p = e;
                if (L > 0) {
                    have = true;
                    tk0 = a0w; tk1 = a1w; tlen = L; tstart = start; traw = (uint32_t)(e - start);
                    break;
                }
            }
            if (!__any(have)) break;
            my_tokens += have ? 1u : 0u;
            emit<CAP, IDX, WIDE>(A, table, R, have, tk0, tk1, tlen, tstart, traw, docid);
        }
    return my_tokens;
}

// ---- UTF-8-exact byte classes for blocks with a non-ASCII byte where the fast path reads (the
// block's two tiles, the first segment of its halo, the byte before it): see k_map's block step.
#define LDS __attribute__((address_space(3)))
// class of codepoint cp: U+0080..07FF and U+2000..20FF from the LDS copy uc, the rest from the table
__device__ __forceinline__ uint32_t uni_class(const LDS uint8_t *uc, uint32_t cp) {
    uint32_t byte;
    if (cp < 0x800u) byte = uc[cp >> 2];
    else if ((cp >> 8) == 0x20u) byte = uc[512u + ((cp & 255u) >> 2)];
    else return mrg_uclass(cp);
    return (byte >> (2u * (cp & 3u))) & 3u;
}
template <int CAP, bool IDX, bool WIDE>
__global__ __launch_bounds__(WG, 1) void k_map(const MapArgs *__restrict__ Ap) {
    // the arguments live in device memory (not the kernarg segment): fields are loaded where they
    // are used instead of being held in SGPRs for the whole kernel
    const MapArgs &A = *Ap;
    // per wave: staged window, 2-segment mask windows, token queue (waves work on their own tiles)
    __shared__ __attribute__((aligned(16))) uint8_t s_win[NW][WIN];
    __shared__ __attribute__((aligned(8))) uint64_t s_mp[NW][NMP];  // W(g)|W(g+1)<<16 | (S(g)|S(g+1)<<16)<<32
    // 8-byte aligned rows: the class fix's compacted decode uses a row as 64 u64 slots between tiles
    __shared__ __attribute__((aligned(8))) uint16_t s_q[NW][QCAP];
    static_assert((QCAP * sizeof(uint16_t)) % 8 == 0 && QCAP * sizeof(uint16_t) >= 64 * 8, "queue rows hold 64 u64 slots");
    // LUT and length masks first in LDS (highest alignment): their base then fits the 16-bit
    // offset field of ds_read, so a lookup needs no separate address add
    // Byte class per byte position p of a dword: s_lut[p][c] = (W | S << 4) << p, one byte per byte
    // value, so the four lookups of a dword OR straight into its nibble pair (no per-byte shift).
    // ASCII entries are the exact classes; every byte >= 0x80 gets W and S both (a pair no ASCII byte
    // has), which marks the block's non-ASCII bytes for the UTF-8 class fix at no cost.  The ASCII
    // half of a table is 128 bytes = 32 dwords, one per LDS bank, and one instruction reads one table:
    // on ASCII text a wave's lookups never conflict (lanes reading the same dword share it)
    __shared__ __attribute__((aligned(1024))) uint8_t s_lut[4][256];
    // v_perm selectors per (key length, 1-byte gap position; 16 = none) over the r-aligned window
    __shared__ __attribute__((aligned(16))) uint32_t s_sel[17 * 17][4];
    // workgroup: combine table + tail-region cursors
    // (the wide map has no table and no tail regions: their LDS holds its bucket cursors and splitters)
    __shared__ KeyPair s_key[WIDE ? 2 : CAP];
    __shared__ unsigned int s_cnt[WIDE ? 2 : CAP];
    __shared__ __attribute__((aligned(16))) unsigned int s_doc[IDX ? CAP : 1];
    __shared__ unsigned long long s_tcur[WIDE ? 1 : MRG_NBUCKET];  // next pool record of (bucket, this WG)
    __shared__ unsigned long long s_tend[WIDE ? 1 : MRG_NBUCKET];  // end of that region
    __shared__ unsigned long long s_tcur16[(IDX || WIDE) ? 1 : MRG_NBUCKET];  // wc: the 16-byte regions
    __shared__ unsigned long long s_tend16[(IDX || WIDE) ? 1 : MRG_NBUCKET];
    __shared__ uint32_t s_hist[WIDE ? 1 : MRG_NBUCKET + 1];
    __shared__ unsigned int s_wcur[WIDE ? MRG_WMAP_MAXB1 : 1];                  // wide: records per L1 bucket
    __shared__ __attribute__((aligned(16))) uint64_t s_wspl[WIDE ? 2 * MRG_WMAP_MAXB1 : 1];  // its splitters
    __shared__ __attribute__((aligned(4))) uint8_t s_wix[WIDE ? MRG_WMAP_IXR * MRG_WIDE_IX1 : 4];
    __shared__ uint32_t s_next, s_ngen;                  // next block of the workgroup's share; list length
    __shared__ uint32_t s_stolen;                        // pool blocks this workgroup's waves have claimed
    __shared__ uint32_t s_pool[NW][3];                   // per wave: its pool chunk [cur, end) past n_static, part | tried << 8
    __shared__ uint32_t s_nuni;                          // non-ASCII tiles tokenized with UTF-8-exact masks
    // the class table's blocks for U+0000..U+07FF (2-byte codepoints: Latin-1, Latin Extended, Greek,
    // Cyrillic, ...) and U+2000..U+20FF (General Punctuation: the quotes and dashes of English text),
    // 2 bits per codepoint; other codepoints read the global table
    __shared__ uint8_t s_uc[9 * 64];
    __shared__ uint32_t s_tot[3];                        // workgroup totals: tokens, tail records, 16-byte ones
    __shared__ unsigned int s_fill;                      // table slots claimed
    __shared__ unsigned int s_lcnt;                      // long-token records (region cursor)
    __shared__ unsigned int s_door[(MRG_MAP_DOOR && !WIDE) ? LdsTable<CAP, IDX>::DW : 1];  // admission bitmap
    static_assert(WIDE || sizeof(s_q) >= CAP * sizeof(uint16_t), "flush ranks reuse the queues");
    static_assert((CAP & (CAP - 1)) == 0 && CAP >= 64 && CAP <= 65536, "2-way sets: NS = CAP / 2 a power of two, ranks in u16");
    static_assert(sizeof(s_door) / sizeof(s_door[0]) >= ((MRG_MAP_DOOR && !WIDE) ? LdsTable<CAP, IDX>::DW : 1u), "doorkeeper words");
    static_assert(!WIDE || (sizeof(s_wcur) / sizeof(s_wcur[0]) == MRG_WMAP_MAXB1 && sizeof(s_wspl) / sizeof(s_wspl[0]) == 2 * MRG_WMAP_MAXB1 &&
                            sizeof(s_wix) == MRG_WMAP_IXR * MRG_WIDE_IX1 && MRG_WIDE_IX1 % 4 == 0),
                  "wide map: cursors, splitters and index rows as the host plan sizes them");
    // the wide map's run-time sizes against those arrays (the host plan keeps R * B1r <= MRG_WMAP_MAXB1
    // and passes an index only when R <= MRG_WMAP_IXR, mrgpu.cpp wide_map_plan; job_map_wide refuses
    // a plan that breaks them before the launch): a launch that still did would return here, uniformly,
    // instead of indexing past LDS
    if constexpr (WIDE) {
        if (A.wR * A.wB1r > (uint32_t)MRG_WMAP_MAXB1 || A.wB1r == 0u || (A.wix && A.wR > (uint32_t)MRG_WMAP_IXR)) return;
    }

    const int tid = threadIdx.x;
    // wave index through readfirstlane: the compiler then knows everything derived from it (tile
    // index, document bounds) is wave-uniform and keeps it in SGPRs
    const int lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    if constexpr (WIDE) {
        const uint32_t nb1 = A.wR * A.wB1r, nsp = 2u * A.wR * (A.wB1r - 1u);
        for (uint32_t b = tid; b < nb1; b += WG) s_wcur[b] = 0;
        for (uint32_t i = tid; i < nsp; i += WG) s_wspl[i] = gp(A.wspl)[i];
        if (A.wix)
            for (uint32_t i = tid; i < A.wR * (MRG_WIDE_IX1 / 4); i += WG)
                reinterpret_cast<uint32_t *>(s_wix)[i] = gp(reinterpret_cast<const uint32_t *>(A.wix))[i];
    }
    for (int i = tid; i < (WIDE ? 2 : CAP); i += WG) {
        s_key[i] = KeyPair{MRG_EMPTY_K0, MRG_EMPTY_K1};
        s_cnt[i] = 0;
        if (IDX) s_doc[i] = MRG_EMPTY_DOC;
    }
    if (MRG_MAP_DOOR && !WIDE)
        for (int i = tid; i < (int)LdsTable<CAP, IDX>::DW; i += WG) s_door[i] = 0;
    for (int b = tid; b < (WIDE ? 0 : MRG_NBUCKET); b += WG) {
        const uint32_t cap = gp(A.bcap)[b];
        const uint64_t base = gp(A.rbase)[b] + (uint64_t)blockIdx.x * cap;
        s_tcur[b] = base;
        s_tend[b] = base + cap;
        if (!IDX) {
            const uint32_t cap16 = gp(A.bcap16)[b];
            const uint64_t base16 = gp(A.rbase16)[b] + (uint64_t)blockIdx.x * cap16;
            s_tcur16[b] = base16;
            s_tend16[b] = base16 + cap16;
        }
    }
    if (tid == 0) {
        s_next = 0;
        s_stolen = 0;
        s_ngen = 0;
        s_nuni = 0;
        s_tot[0] = 0;
        s_tot[1] = 0;
        s_tot[2] = 0;
        s_fill = 0;
        s_lcnt = 0;
    }
    // (strided: a workgroup of fewer than 1024 threads -- the occupancy-sweep builds -- fills them too)
    for (int i = tid; i < 9 * 64; i += WG) {
        const uint32_t blk = i < 512 ? (uint32_t)i >> 6 : 0x20u;
        s_uc[i] = c_uclass_stage2[c_uclass_stage1[blk] * 64u + ((uint32_t)i & 63u)];
    }
    for (int i = tid; i < 1024; i += WG) {
        const uint32_t v = (uint32_t)i & 255u, c = mrg_uclass(v & 127u);
        const uint32_t ws = v >= 128u ? 0x11u : ((c == MRG_CLS_W ? 1u : 0u) | (c == MRG_CLS_S ? 0x10u : 0u));
        s_lut[i >> 8][v] = (uint8_t)(ws << (i >> 8));
    }
    auto zmask = [](uint32_t L, uint32_t j) {  // word j, byte p (p = 0 least significant) holds key byte 4j + 3 - p
        uint32_t m = 0;
        for (uint32_t p = 0; p < 4; ++p)
            if (4u * j + 3u - p >= L) m |= 0xFFu << (8u * p);
        return m;
    };
    for (int i = tid; i < 17 * 17 * 4; i += WG) {
        // key byte 4j + 3 - p comes from aligned-window byte 4j + 3 - p (+ 1 from the gap on); bytes
        // at or past the key length select the constant 0 (v_perm selector 0x0C)
        const uint32_t L = (uint32_t)i / 68u, g = ((uint32_t)i / 4u) % 17u, j = (uint32_t)i & 3u;
        const uint32_t zm = zmask(L, j), gm = zmask(g, j);
        s_sel[L * 17u + g][j] = ((0x00010203u + (gm & 0x01010101u)) & ~zm) | (0x0C0C0C0Cu & zm);
    }
    LdsTable<CAP, IDX> table{s_key, s_cnt, s_doc, s_door, &s_fill};
    const TailRegions tails{s_tcur, s_tend, s_tcur16, s_tend16, &s_lcnt, s_wcur, s_wspl, A.wix ? s_wix : nullptr};
    uint32_t my_tokens = 0;
    // uniform job parameters used in the hot loop, read once
    // ablation knobs (MRG_ABLATE, timing only) exist in -DMRG_MAP_ABLATION builds; in the product
    // build abl is the constant 0, so no branch, mask or SGPR of the hot loop is spent on them
#ifdef MRG_MAP_ABLATION
    const uint32_t abl = A.ablate;
#else
    constexpr uint32_t abl = MRG_MAP_ABL_CONST;
#endif
    const uint32_t hbits = A.hash_bits;
    GAS uint64_t *const pool = gp(A.pool);
    GAS uint64_t *const pool16 = gp(A.pool16);
    uint8_t *win = s_win[wv];
    uint64_t *mp = s_mp[wv];
    uint16_t *queue = s_q[wv];
    __syncthreads();

    // Tile staging for the walkers (deferred non-ASCII tiles): 16-byte vectors j relative to At - 16:
    // j = 0 the bytes before the tile, j = 1..64 the tile's segments, j = 65..68 the halo.  Lane l
    // loads vector 1 + l; lanes 0..4 also vectors 0 and 65..68.  Only vectors in [v0, v1) are read.
    const uint32_t j0 = 1u + (uint32_t)lane;
    const uint32_t j1 = lane == 0 ? 0u : 64u + (uint32_t)lane;
    const bool has1 = lane < 5;
    auto load = [&](const TileInfo &t, uint4 &p0, uint4 &p1) {
        const GAS u32x4 *src = reinterpret_cast<const GAS u32x4 *>(gp(A.in) + (t.At - (uint64_t)BEHIND));
        u32x4 v0 = {0, 0, 0, 0}, v1 = {0, 0, 0, 0};
        if (j0 >= t.v0 && j0 < t.v1) v0 = src[j0];
        if (has1 && j1 >= t.v0 && j1 < t.v1) v1 = src[j1];
        p0 = uint4{v0.x, v0.y, v0.z, v0.w};
        p1 = uint4{v1.x, v1.y, v1.z, v1.w};
    };
    // A 2 KiB block in registers: lane l holds bytes [Ab + 1024 j + 16 l, +16) in v[j]; e = the 16
    // bytes before the block on lane 0, the 64-byte halo after it on lanes 1..4.  The three loads are
    // unconditional (no branch for the scheduler to wait inside): an out-of-range lane reads a
    // clamped in-range vector instead.  Its bytes are never used as text: classify() turns every
    // byte outside the document into White_Space, and keys only come from bytes inside it.
    struct Blk {
        uint4 v0, v1, e;
    };
#ifdef MRG_MAP_ABLATION
    BlkInfo first_blk{};  // ablate & 8 (timing only): every block re-reads the wave's first block
#endif
    auto load_blk = [&](const BlkInfo &b0, Blk &X) {
#ifdef MRG_MAP_ABLATION
        const BlkInfo &b = (abl & 8u) ? first_blk : b0;  // a real block: its own base and bounds
#else
        const BlkInfo &b = b0;
#endif
        const GAS uint8_t *src = gp(A.in) + (b.Ab - (uint64_t)BEHIND);
        auto ld = [&](uint32_t idx) -> uint4 {
            const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const GAS u32x4 *>(src + 16u * min(max(idx, b.v0), b.v1 - 1u)));
            return uint4{t.x, t.y, t.z, t.w};
        };
        X.v0 = ld(1u + (uint32_t)lane);
        X.v1 = ld(65u + (uint32_t)lane);
        X.e = ld(lane == 0 ? 0u : 128u + (uint32_t)lane);
    };

    // Work split: workgroup w owns blocks [wlo_b, whi_b) (equal shares of the first n_static); its
    // waves take the next block from an LDS counter, so a wave that the SIMD's age-ordered issue leaves
    // behind simply takes fewer blocks (a static per-wave split left the youngest waves finishing last).
    // The blocks past n_static are a pool the waves of workgroups done with their share take from
    // (r06: workgroups ran 7.14-7.58 ms on equal shares of C3, the launch lasting as long as the
    // slowest), MRG_MAP_STEAL_K at a time from one of 8 part counters, within the workgroup's budget.
    const uint64_t ns = A.n_static;  // blocks in equal shares (of A.n_chunks)
    const uint64_t wlo_b = ns * blockIdx.x / gridDim.x, whi_b = ns * (blockIdx.x + 1) / gridDim.x;
    // non-ASCII tiles: appended to this workgroup's list (absolute tile index: block * NSUB + tile),
    // processed after the main loop by all 16 waves
    GAS uint32_t *glist = gp(A.gbits) + (uint64_t)blockIdx.x * A.kwords;

    // one block: masks of its 1 KiB tiles up front, then tile by tile through the
    // wave's LDS window
    // phase clocks (MRG_PROF only; wave-uniform): 0 wait for the block's loads, 1 classify,
    // 2 stage + scan + queue, 3 token rounds, 4 slow tokens, 5 non-ASCII tiles, 6 flush
    // (a diagnostic build only: -DMRG_MAP_PROF; the accumulators would otherwise take 16 SGPRs of
    // a kernel that already spills SGPRs)
#ifdef MRG_MAP_PROF
    const bool P = A.prof != nullptr;
    uint64_t pacc[7] = {0, 0, 0, 0, 0, 0, 0}, tl = P ? clock64() : 0;
    const uint64_t wg_t0 = wall_clock64();  // workgroup start/end (100 MHz): load balance across CUs
    unsigned long long ftv[5] = {0, 0, 0, 0, 0};   // flush step ends (wall clock, workgroup thread 0)
#define MRG_FT(i)                                   \
    if (P && tid == 0) ftv[i] = wall_clock64();
#define MRG_PT(i)                          \
    if (P) {                               \
        const uint64_t t_ = clock64();     \
        pacc[i] += t_ - tl;                \
        tl = t_;                           \
    }
#else
#define MRG_PT(i)
#define MRG_FT(i)
#endif
    // A token of the wave's queue: entry q (of total) holds its start s (tile offset); its raw
    // length, \w span and deleted bytes come from one 8-byte mask-pair read, its key bytes from the
    // window.  fast: a key of <= 16 bytes ending inside the 2-segment window; slow: the rest (the
    // exact walker).  Returns the deleted-byte runs still to squeeze out (more than one).
    auto extract = [&](uint32_t q, uint32_t sraw, uint32_t total, bool &fast, bool &slow, uint32_t &s,
                       uint64_t &tk0, uint64_t &tk1) -> uint32_t {
        const bool act = q < total;
        s = act ? sraw : 0u;
        const uint64_t mw = mp[s >> 4];
        const uint32_t Wp = (uint32_t)mw, Sp = (uint32_t)(mw >> 32);
        const uint32_t i = s & 15u;
        const uint32_t Sr = Sp >> i;
        const uint32_t n = (uint32_t)__builtin_ctz(Sr | 0x80000000u);  // raw length (if Sr != 0)
        const bool ended = Sr != 0u;                                     // end inside the 2 segments
        const uint32_t w = __builtin_amdgcn_ubfe(Wp, i, n);              // \w bits of the raw token
        const uint32_t first = (uint32_t)__builtin_ctz(w | 0x80000000u);
        const uint32_t last = 31u - (uint32_t)__builtin_clz(w | 1u);
        const uint32_t span = last - first + 1u;
        // bitwise on purpose: lane masks combined by SALU, no per-lane selects
        const bool wz = w == 0u, big = span > 16u;
        fast = act & ended & !wz & !big;
        slow = act & (!ended | (!wz & big));
        // deleted bytes inside the token ("don't"): one 1-byte gap is folded into the selectors
        // below (key bytes from the gap on come from one window byte later); tokens with more
        // gaps squeeze them out afterwards
        const uint32_t gaps = fast ? (~(w >> first) & ((1u << span) - 1u)) : 0u;
        const bool one_gap = gaps != 0u && (gaps & (gaps - 1u)) == 0u;
        const uint32_t ga = one_gap ? (uint32_t)__builtin_ctz(gaps) : 16u;
        uint32_t tlen = one_gap ? span - 1u : span;
        // key bytes of the window from s + first, big-endian packed, zero padded: output byte p
        // of word j is key byte 4j + 3 - p (selector r + 3 - p [+ 1 past the gap], 0x0C = zero)
        // the 17 window bytes from the key's first byte as five dwords: one unaligned 16-byte
        // LDS read and one 4-byte read (gfx950 runs in unaligned access mode: no dword
        // alignment, no v_alignbyte), then one selector word per output word
        const uint32_t off = (uint32_t)BEHIND + s + first;
        const uint32_t *win32 = reinterpret_cast<const uint32_t *>(win);
        const uint32_t dw = off >> 2, r = off & 3u;
        const uint32_t d0 = win32[dw], d1 = win32[dw + 1], d2 = win32[dw + 2], d3 = win32[dw + 3],
                       d4 = win32[dw + 4];
        const u32x4 sl = *reinterpret_cast<const u32x4 *>(s_sel[(fast ? tlen : 0u) * 17u + ga]);
        const uint32_t a0 = __builtin_amdgcn_alignbyte(d1, d0, r), a1 = __builtin_amdgcn_alignbyte(d2, d1, r),
                       a2 = __builtin_amdgcn_alignbyte(d3, d2, r), a3 = __builtin_amdgcn_alignbyte(d4, d3, r),
                       a4 = __builtin_amdgcn_alignbyte(0u, d4, r);
        const uint32_t o0 = __builtin_amdgcn_perm(a1, a0, sl.x);
        const uint32_t o1 = __builtin_amdgcn_perm(a2, a1, sl.y);
        const uint32_t o2 = __builtin_amdgcn_perm(a3, a2, sl.z);
        const uint32_t o3 = __builtin_amdgcn_perm(a4, a3, sl.w);
        tk0 = ((uint64_t)o0 << 32) | o1;
        tk1 = ((uint64_t)o2 << 32) | o3;
        return one_gap ? 0u : gaps;  // gaps still to squeeze out
    };
    // squeeze out the remaining gaps (more than one deleted run inside the token; rare)
    auto squeeze = [](uint32_t mgaps, uint64_t &tk0, uint64_t &tk1) {
        while (mgaps) {
            const uint32_t ga2 = (uint32_t)__builtin_ctz(mgaps);          // gap start (key byte)
            const uint32_t gl = (uint32_t)__builtin_ctz(~(mgaps >> ga2)); // gap length
            const uint32_t sh = 8u * gl;                                  // 8..120 bits
            // shifted = (tk0:tk1) << sh; keep the top ga2 bytes, take the rest from shifted
            uint64_t s0v, s1v;
            if (sh >= 64u) { s0v = tk1 << (sh - 64u); s1v = 0; }
            else { s0v = (tk0 << sh) | (tk1 >> (64u - sh)); s1v = tk1 << sh; }
            const uint32_t kb = 8u * ga2;                                 // kept bits
            const uint64_t k0m = kb >= 64u ? ~0ull : (kb ? ~0ull << (64u - kb) : 0ull);
            const uint64_t k1m = kb <= 64u ? 0ull : ~0ull << (128u - kb);
            tk0 = (tk0 & k0m) | (s0v & ~k0m);
            tk1 = (tk1 & k1m) | (s1v & ~k1m);
            mgaps = (mgaps >> (ga2 + gl)) << ga2;
        }
    };

    // A deferred slow token through the tile's byte classes (r04): the mask pairs mp[] hold W16 / S16
    // of every segment of the tile, exact for UTF-8 too (pair k = segments k and k + 1, so the last
    // pair's high halves are the first halo segment), and the window holds its bytes -- the token's
    // end and key need no codepoint decoding: the key is the W bytes before the first S byte.  s = the
    // token's tile offset, nseg = the tile's segments.  False when the token runs past the first halo
    // segment (then the codepoint walker).
    auto mask_walk = [&](uint32_t s, uint32_t nseg, uint64_t &tk0, uint64_t &tk1, uint32_t &tlen,
                         uint32_t &traw) -> bool {
        tk0 = 0;
        tk1 = 0;
        tlen = 0;
        const uint32_t *win32 = reinterpret_cast<const uint32_t *>(win);
        uint32_t i = s & 15u;
        for (uint32_t seg = s >> 4; seg <= nseg; ++seg, i = 0) {
            const uint64_t mw = mp[seg < nseg ? seg : nseg - 1u];
            const uint32_t sh = seg < nseg ? 0u : 16u;
            uint32_t W = ((((uint32_t)mw >> sh) & 0xFFFFu) >> i) << i;
            const uint32_t S = ((((uint32_t)(mw >> 32) >> sh) & 0xFFFFu) >> i) << i;
            const uint32_t e = S ? (uint32_t)__builtin_ctz(S) : 16u;
            W &= (1u << e) - 1u;
            // key bytes (only the first 16 are packed): each run of W bytes as one selector load (the
            // fast path's), shifted behind the bytes so far
            while (W && tlen < 16u) {
                const uint32_t b = (uint32_t)__builtin_ctz(W);
                const uint32_t r = (uint32_t)__builtin_ctz(~(W >> b));  // run length (<= 16 - b)
                W &= ~(((1u << r) - 1u) << b);
                const uint32_t off = (uint32_t)BEHIND + 16u * seg + b;
                const uint32_t dw = off >> 2, ra = off & 3u;
                const uint32_t d0 = win32[dw], d1 = win32[dw + 1], d2 = win32[dw + 2], d3 = win32[dw + 3],
                               d4 = win32[dw + 4];
                const u32x4 sl = *reinterpret_cast<const u32x4 *>(s_sel[r * 17u + 16u]);
                const uint32_t a0 = __builtin_amdgcn_alignbyte(d1, d0, ra), a1 = __builtin_amdgcn_alignbyte(d2, d1, ra),
                               a2 = __builtin_amdgcn_alignbyte(d3, d2, ra), a3 = __builtin_amdgcn_alignbyte(d4, d3, ra),
                               a4 = __builtin_amdgcn_alignbyte(0u, d4, ra);
                const uint64_t v0 = ((uint64_t)__builtin_amdgcn_perm(a1, a0, sl.x) << 32) | __builtin_amdgcn_perm(a2, a1, sl.y);
                const uint64_t v1 = ((uint64_t)__builtin_amdgcn_perm(a3, a2, sl.z) << 32) | __builtin_amdgcn_perm(a4, a3, sl.w);
                // (v0:v1) >> 8 * tlen
                const uint32_t ks = 8u * tlen;
                if (ks == 0u) {
                    tk0 |= v0;
                    tk1 |= v1;
                } else if (ks < 64u) {
                    tk0 |= v0 >> ks;
                    tk1 |= (v1 >> ks) | (v0 << (64u - ks));
                } else {
                    tk1 |= v0 >> (ks - 64u);
                }
                tlen += r;
            }
            tlen += (uint32_t)__builtin_popcount(W);
            if (S) {
                traw = 16u * seg + e - s;
                return true;
            }
        }
        return false;
    };

    auto process_blk = [&](const BlkInfo &I, const Blk &X, uint64_t cblk, auto &&mid) {
        const uint64_t Ab = I.Ab, doc_lo = I.doc_lo, doc_hi = I.doc_hi;
        const uint32_t docid = I.docid;
        // classify segment [B, B + 16) (relative to Ab) into W16 | S16 << 16; bytes outside the
        // document count as White_Space (exact for every staged byte: no window cut)
        const uint32_t lo_rel = doc_lo > Ab ? (uint32_t)(doc_lo - Ab) : 0u;
        const uint32_t hi_rel = (uint32_t)umin64(doc_hi - Ab, (uint64_t)(BLK + HALO));
        auto classify = [&](const uint4 &x, uint32_t B) -> uint32_t {
            // all 16 lookups in flight before the first use (one LDS wait per segment); byte b of a
            // dword reads table b, whose entries are already shifted to bit b (W) and 4 + b (S)
            uint32_t e[16];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t w = k == 0 ? x.x : (k == 1 ? x.y : (k == 2 ? x.z : x.w));
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    e[4 * k + b] = s_lut[b][b == 0 ? (w & 0xFFu) : (b == 3 ? w >> 24 : __builtin_amdgcn_ubfe(w, 8 * b, 8))];
            }
            // nibbles: W of bytes 0-3, S of bytes 0-3, W of bytes 4-7, ... (byte i: bit i % 4):
            // dword k's byte of y is the OR of its four lookups
            uint32_t yk[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) yk[k] = e[4 * k] | e[4 * k + 1] | e[4 * k + 2] | e[4 * k + 3];
            const uint32_t y = (yk[0] | (yk[1] << 8)) | ((yk[2] | (yk[3] << 8)) << 16);
            const uint32_t t = y & 0x0F0F0F0Fu, u = (y >> 4) & 0x0F0F0F0Fu;
            // bytes 0 and 2 of t | t >> 4: W of bytes 0-7 and 8-15 (u: S)
            const uint32_t m = __builtin_amdgcn_perm(u | (u >> 4), t | (t >> 4), 0x06040200u);  // W16 | S16 << 16
            const uint32_t lo_inv = lo_rel > B ? min(lo_rel - B, 16u) : 0u;
            const uint32_t hi_ok = B < hi_rel ? min(hi_rel - B, 16u) : 0u;
            const uint32_t valid = ((1u << hi_ok) - 1u) & ~((1u << lo_inv) - 1u);
            return (m & (valid | (valid << 16))) | ((~valid & 0xFFFFu) << 16);
        };
        auto na = [](const uint4 &x) { return ((x.x | x.y | x.z | x.w) & 0x80808080u) != 0u; };
        const uint32_t l16 = (uint32_t)lane * SEG;
        uint32_t m0 = classify(X.v0, l16), m1 = classify(X.v1, 1024u + l16);
        // the first halo segment (lane 1's e) by 16 lanes, one byte each, through two ballots
        uint32_t mh;
        {
            const uint32_t e0 = lane_u32(X.e.x, 1), e1 = lane_u32(X.e.y, 1), e2 = lane_u32(X.e.z, 1),
                           e3 = lane_u32(X.e.w, 1);
            const uint32_t k = (uint32_t)lane & 15u;
            const uint32_t dwv = k < 8u ? (k < 4u ? e0 : e1) : (k < 12u ? e2 : e3);
            const uint32_t cl = s_lut[0][__builtin_amdgcn_ubfe(dwv, 8u * (k & 3u), 8)];
            const bool in = (uint32_t)BLK + k < hi_rel;  // bytes past the document are White_Space
            const uint32_t wm = (uint32_t)__ballot(lane < 16 && in && (cl & 1u));
            const uint32_t sm = (uint32_t)__ballot(lane < 16 && (!in || (cl & 0x10u)));
            mh = (wm & 0xFFFFu) | (sm << 16);
        }
        const bool n0 = na(X.v0), n1 = na(X.v1), ne = na(X.e);
        // class of the byte before the block (lane 0's e, byte 15)
        uint32_t prev_blk =
            Ab > doc_lo ? (uint32_t)(s_lut[0][lane_u32(X.e.w, 0) >> 24] >> 4) & 1u : 1u;
        // A non-ASCII byte where the fast path reads (either tile, the first halo segment, the bytes
        // before the block): the LUT classes of the non-ASCII bytes are replaced by UTF-8-exact ones,
        // after which both tiles are tokenized exactly like ASCII tiles -- every byte of a codepoint
        // carries its class, so the W / S masks mean the same.  Invalid UTF-8 defers the block's tiles
        // to generic_tile after the main loop (which reports the first bad byte).
        bool defer_blk = false;
        if (!(abl & 256u) && !(MRG_MAP_ABL_CONST & 0x20000u) && __any(n0 || n1 || (lane <= 1 && ne))) {
#ifdef MRG_MAP_NO_UNI
            defer_blk = true;  // A/B builds only: every such block to the exact walker, as in r03
#else
            // UTF-8-exact classes in registers (r05): every lane decodes the codepoints whose leads lie
            // in its own segments, straight from the segment's four dwords and the next segment's first
            // (DPP) -- no LDS window.  One loop over the lane's leads, both segments per trip (the trip
            // count is the busiest lane's lead count: about 1.6 per block on English text, whose
            // non-ASCII codepoints are sparse), unless a lane holds two or more: then the compacted
            // decode below takes one trip (MRG_MAP_CMPT).  A lead's bytes are checked by the
            // decode (continuation bytes, overlongs, surrogates, range); a codepoint's last bytes may lie in
            // the next segment (spilled by DPP).  Every non-ASCII byte must be covered by a decoded
            // codepoint, else the block holds invalid UTF-8 and is deferred.  (r04 compacted the leads
            // into the wave's queue and decoded one per lane from the staged window: two stagings,
            // two queue fills and two divergent read-backs per block, and a queue that invalid input
            // with more than 528 leads per tile could overflow.)
            const int64_t dlo = (int64_t)(doc_lo - Ab);  // two's complement (see lo below)
            // the document in block offsets: lo in [-16, 16), hi in (0, 2112].  (A select on
            // doc_lo > Ab lost its first case in the compiled code: keep a clamped signed difference.)
            const int lo = (int)(dlo < -(int64_t)BEHIND ? -(int64_t)BEHIND : dlo);
            const int hi = (int)umin64(doc_hi - Ab, (uint64_t)(BLK + HALO));
            const LDS uint8_t *uc = (const LDS uint8_t *)s_uc;
            bool bad = false;
            auto hb = [](uint32_t d) { return ((((d & 0x80808080u) >> 7) * 0x00204081u) >> 21) & 0xFu; };
            // the non-ASCII bytes inside the document: W and S both set by the LUT (bytes outside the
            // document were made White_Space only); of those, the codepoint leads (>= 0xC0)
            auto nam_of = [](uint32_t m) { return m & (m >> 16) & 0xFFFFu; };
            auto leads = [&](const uint4 &x, uint32_t nam) {
                return (hb(x.x & (x.x << 1)) | (hb(x.y & (x.y << 1)) << 4) | (hb(x.z & (x.z << 1)) << 8) |
                        (hb(x.w & (x.w << 1)) << 12)) & nam;
            };
            const uint32_t nam0 = nam_of(m0), nam1 = nam_of(m1), namh_w = nam_of(mh);  // mh: wave-uniform
            const uint32_t ld0 = leads(X.v0, nam0), ld1 = leads(X.v1, nam1);
            uint4 xh{0u, 0u, 0u, 0u};
            uint32_t namh = 0u, ldh = 0u;
            if (namh_w) {  // the first halo segment (lane 63's) holds non-ASCII bytes (wave-uniform)
                xh = uint4{lane_u32(X.e.x, 1), lane_u32(X.e.y, 1), lane_u32(X.e.z, 1), lane_u32(X.e.w, 1)};
                if (lane == 63) {
                    namh = namh_w;
                    ldh = leads(xh, namh);
                }
            }
            // the byte before the block (inside the document and not ASCII): the lead of its codepoint,
            // 1..4 bytes back (wave-uniform)
            const uint32_t before = lane_u32(X.e.w, 0);  // block bytes -4..-1
            int pbp = 0;
            bool has_b = false;
            if (dlo < 0 && (before >> 24) >= 0x80u) {
                uint32_t bb = before >> 24;
                pbp = -1;
                for (int k = 2; k <= 4 && (bb & 0xC0u) == 0x80u; ++k) {
                    bb = (before >> (8 * (4 - k))) & 0xFFu;
                    pbp = -k;
                }
                if (bb < 0xC0u || pbp < lo) bad = true;
                else has_b = true;
            }
            // the 4 bytes after each segment: the next lane's first dword (lane 63: tile 1's first
            // segment after tile 0, the first halo segment after tile 1); after the halo segment, lane
            // 2's e (the halo's next 16 bytes)
            const uint32_t v1_first = lane_u32(X.v1.x, 0), halo_next = lane_u32(X.e.x, 2);
            uint32_t nA = from_next_lane(X.v0.x), nB = from_next_lane(X.v1.x);
            if (lane == 63) {
                nA = v1_first;
                nB = xh.x;
            }
            // one codepoint whose lead is byte p of the 20-byte window d0..d4 starting at block offset so:
            // W / S / covered-byte masks over the window (bits 16..19 spill into the next segment)
            auto dec = [&](uint32_t p, uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3, uint32_t d4, int so,
                           uint32_t &W, uint32_t &S, uint32_t &C) {
                const uint32_t k = p >> 2;
                const uint32_t a = (k & 2u) ? ((k & 1u) ? d3 : d2) : ((k & 1u) ? d1 : d0);
                const uint32_t b = (k & 2u) ? ((k & 1u) ? d4 : d3) : ((k & 1u) ? d2 : d1);
                const uint32_t w = __builtin_amdgcn_alignbyte(b, a, p & 3u);
                auto rd = [&](uint64_t x) -> uint32_t { return (w >> (8u * (uint32_t)x)) & 0xFFu; };
                uint32_t cp = 0, raw;
                const int n = mrg_utf8_decode(rd, 0ull, (uint64_t)min(hi - (so + (int)p), 4), &cp, &raw);
                bad |= n == 0;
                const uint32_t span = ((1u << n) - 1u) << p;
                const uint32_t cl = uni_class(uc, cp);
                C |= span;
                W |= cl == MRG_CLS_W ? span : 0u;
                S |= cl == MRG_CLS_S ? span : 0u;
            };
            uint32_t W0 = 0, S0 = 0, C0 = 0, W1 = 0, S1 = 0, C1 = 0;
            uint32_t mAB0 = (MRG_MAP_ABL_CONST & 0x10000u) ? 0u : (ld0 | (ld1 << 16));
#if MRG_MAP_CMPT
            // a lane with two or more leads (about 6 blocks in 10 of English text: one codepoint per
            // ~190 bytes, 32 bytes per lane) would cost the whole wave a second decode trip.  Instead
            // the block's leads are compacted, one per lane (a wave prefix sum of the lead counts):
            // the owner writes each lead's 4 bytes and its byte budget to the wave's token queue (free
            // between tiles), lanes 0..T-1 decode one codepoint each, and the owners read the results
            // back (length | W << 3 | S << 4; length 0 = invalid).
            {
                const uint32_t c = (uint32_t)__builtin_popcount(mAB0);
                if (__any(c >= 2u)) {
                    const uint32_t incl = wave_incl_scan(c);
                    const uint32_t T = lane_u32(incl, 63);
                    if (T <= 64u) {
                        LDS uint64_t *slot = (LDS uint64_t *)queue;
                        wave_sync_lds();
                        uint32_t pos = incl - c;
                        for (uint32_t m = mAB0; m;) {
                            const uint32_t q = (uint32_t)__builtin_ctz(m);
                            m &= m - 1u;
                            const bool sb = q >= 16u;
                            const uint32_t p = q & 15u, k = p >> 2;
                            const uint32_t d0 = sb ? X.v1.x : X.v0.x, d1 = sb ? X.v1.y : X.v0.y,
                                           d2 = sb ? X.v1.z : X.v0.z, d3 = sb ? X.v1.w : X.v0.w, d4 = sb ? nB : nA;
                            const uint32_t a = (k & 2u) ? ((k & 1u) ? d3 : d2) : ((k & 1u) ? d1 : d0);
                            const uint32_t b = (k & 2u) ? ((k & 1u) ? d4 : d3) : ((k & 1u) ? d2 : d1);
                            const int so = (sb ? 1024 : 0) + (int)l16 + (int)p;
                            slot[pos++] = (uint64_t)__builtin_amdgcn_alignbyte(b, a, p & 3u) | ((uint64_t)(uint32_t)min(hi - so, 4) << 32);
                        }
                        wave_sync_lds();
                        if ((uint32_t)lane < T) {
                            const uint64_t s = slot[lane];
                            const uint32_t sw = (uint32_t)s;
                            auto rd = [&](uint64_t x) -> uint32_t { return (sw >> (8u * (uint32_t)x)) & 0xFFu; };
                            uint32_t cp = 0, raw;
                            const uint32_t n = (uint32_t)mrg_utf8_decode(rd, 0ull, s >> 32, &cp, &raw);
                            const uint32_t cl = uni_class(uc, cp);
                            ((LDS uint32_t *)slot)[2 * lane] =
                                n | (cl == MRG_CLS_W ? 8u : 0u) | (cl == MRG_CLS_S ? 16u : 0u);
                        }
                        wave_sync_lds();
                        pos = incl - c;
                        for (uint32_t m = mAB0; m;) {
                            const uint32_t q = (uint32_t)__builtin_ctz(m);
                            m &= m - 1u;
                            const uint32_t r = ((const LDS uint32_t *)slot)[2 * pos++];
                            const uint32_t n = r & 7u;
                            bad |= n == 0u;
                            const uint32_t span = ((1u << n) - 1u) << (q & 15u);
                            const uint32_t w = (r & 8u) ? span : 0u, sm = (r & 16u) ? span : 0u;
                            if (q >= 16u) {
                                W1 |= w; S1 |= sm; C1 |= span;
                            } else {
                                W0 |= w; S0 |= sm; C0 |= span;
                            }
                        }
                        mAB0 = 0u;
                    }
                }
            }
#endif
            // one codepoint per lane and trip, the lane's two segments' leads in one mask (non-ASCII
            // text is sparse: most lanes have none, a few one)
            for (uint32_t mAB = mAB0; __any(mAB != 0u);) {
                if (mAB) {
                    const uint32_t q = (uint32_t)__builtin_ctz(mAB);
                    mAB &= mAB - 1u;
                    const bool sb = q >= 16u;
                    uint32_t w = 0, sm = 0, c = 0;
                    dec(q & 15u, sb ? X.v1.x : X.v0.x, sb ? X.v1.y : X.v0.y, sb ? X.v1.z : X.v0.z,
                        sb ? X.v1.w : X.v0.w, sb ? nB : nA, (sb ? 1024 : 0) + (int)l16, w, sm, c);
                    if (sb) {
                        W1 |= w; S1 |= sm; C1 |= c;
                    } else {
                        W0 |= w; S0 |= sm; C0 |= c;
                    }
                }
            }
            // lane 0: the codepoint holding the byte before the block (window = the 16 bytes before it +
            // the block's first 4, lead at 16 + pbp); lane 63: the first halo segment's leads
            uint32_t WE = 0, SE = 0, CE = 0;
            {
                const bool l0 = lane == 0;
                uint32_t mE = l0 ? (has_b ? 1u << (16 + pbp) : 0u) : ldh;
                const uint4 xe = l0 ? X.e : xh;
                const uint32_t ne = l0 ? X.v0.x : halo_next;
                const int soe = l0 ? -16 : BLK;
                while (__any(mE != 0u)) {
                    if (mE) {
                        const uint32_t p = (uint32_t)__builtin_ctz(mE);
                        mE &= mE - 1u;
                        dec(p, xe.x, xe.y, xe.z, xe.w, ne, soe, WE, SE, CE);
                    }
                }
            }
            uint32_t bsp = 0, pb_l = prev_blk, Wh = 0, Sh = 0, Ch = 0;
            // spills (C | W << 4 | S << 8 of bits 16..18) into the next segment: lane l+1, tile 1's lane
            // 0 after tile 0's lane 63, the halo segment after tile 1's lane 63 (same lane)
            auto pack = [](uint32_t W, uint32_t S, uint32_t C) { return (C >> 16) | ((W >> 16) << 4) | ((S >> 16) << 8); };
            if (lane == 0 && has_b) {
                bad |= (CE & 0x8000u) == 0u;  // the codepoint must reach byte -1
                bsp = pack(WE, SE, CE);
                pb_l = (SE >> 15) & 1u;
            }
            if (lane == 63) {
                Wh = WE;
                Sh = SE;
                Ch = CE;
            }
            const uint32_t sp0 = pack(W0, S0, C0), sp1 = pack(W1, S1, C1);
            uint32_t in0 = from_prev_lane(sp0), in1 = from_prev_lane(sp1);
            const uint32_t sp0_last = lane_u32(sp0, 63);
            if (lane == 0) {
                in0 = bsp;
                in1 = sp0_last;
            }
            auto fix = [&](uint32_t m, uint32_t nam, uint32_t W, uint32_t S, uint32_t C, uint32_t in) -> uint32_t {
                W = (W | ((in >> 4) & 0xFu)) & 0xFFFFu;
                S = (S | ((in >> 8) & 0xFu)) & 0xFFFFu;
                C = (C | (in & 0xFu)) & 0xFFFFu;
                if (!(MRG_MAP_ABL_CONST & 0x10000u)) bad |= C != nam;   // (0x10000: timing only, no decode)
                return ((m & 0xFFFFu & ~nam) | W) | ((((m >> 16) & ~nam) | S) << 16);
            };
            m0 = fix(m0, nam0, W0, S0, C0, in0);
            m1 = fix(m1, nam1, W1, S1, C1, in1);
            uint32_t mh_l = mh;
            if (lane == 63) mh_l = fix(mh, namh, Wh, Sh, Ch, sp1);
            mh = lane_u32(mh_l, 63);
            prev_blk = lane_u32(pb_l, 0);
            defer_blk = __any(bad);
            if (!defer_blk && lane == 0) atomicAdd(&s_nuni, Ab + (uint64_t)TILE < doc_hi ? 2u : 1u);
#endif
        }
        MRG_PT(1);
        // the next block's registers are waited for HERE, before this block's tail stores are
        // issued: vmcnt also counts stores, so a wait placed after them would wait for their
        // acknowledgements too
        mid();
        MRG_PT(0);
        if (defer_blk) {  // recorded; processed after the main loop
            if (lane == 0) {
                for (uint32_t j = 0; j < NSUB && Ab + (uint64_t)j * TILE < doc_hi; ++j) {
                    const uint32_t k = atomicAdd(&s_ngen, 1u);
                    glist[k] = (uint32_t)(cblk * NSUB + j);
                }
            }
            return;
        }
        if (abl & 32u) {  // timing only: classification alone
            my_tokens += (m0 ^ m1 ^ mh ^ prev_blk) & 1u;
            return;
        }

#pragma unroll
        for (uint32_t j = 0; j < NSUB; ++j) {
            const uint64_t At = Ab + (uint64_t)j * TILE;
            if (At >= doc_hi) break;
            const bool last = j == NSUB - 1;
            const uint32_t mlut = j == 0 ? m0 : m1;
            const uint32_t mprev = m0;
            const uint64_t t1 = umin64(At + (uint64_t)TILE, doc_hi);
            const uint64_t whi = umin64(t1 + (uint64_t)HALO, doc_hi);
            const uint64_t wbase = At - (uint64_t)BEHIND;
            // stage the tile and its 64-byte halo (the previous tile's readers are done: program order)
            wave_sync_lds();
            reinterpret_cast<uint4 *>(win)[1 + lane] = j == 0 ? X.v0 : X.v1;
            if (j == 0 ? lane < 4 : (lane >= 1 && lane < 5))
                reinterpret_cast<uint4 *>(win)[65 + (j == 0 ? lane : lane - 1)] = j == 0 ? X.v1 : X.e;
            // masks: this lane's segment and the next one (lane 63: the first halo segment)
            const uint32_t m = mlut;
            uint32_t mn = from_next_lane(m);
            if (lane == 63) mn = !last ? lane_u32(m1, 0) : mh;
            // token starts of this lane's segment: the previous byte's class from lane l-1 (lane 0:
            // the previous tile's last byte); each start gets a queue slot by a wave prefix sum
            uint32_t prev = from_prev_lane(m) >> 31;
            if (lane == 0) prev = j == 0 ? prev_blk : (lane_u32(mprev, 63) >> 31);
            const uint32_t Wpair = (m & 0xFFFFu) | (mn << 16);
            const uint32_t Spair = (m >> 16) | (mn & 0xFFFF0000u);
            mp[lane] = (uint64_t)Wpair | ((uint64_t)Spair << 32);
            const uint32_t S = m >> 16;
            uint32_t st = ~S & ((S << 1) | prev) & 0xFFFFu;
            if (l16 >= (uint32_t)(t1 - At)) st = 0;
            const uint32_t cnt = __builtin_popcount(st);
            const uint32_t incl = wave_incl_scan(cnt);
            uint32_t pos = incl - cnt;
            if (abl & 64u) {  // timing only: no queue writes, no tokens
                my_tokens += st & 1u;
                st = 0;
            }
            while (st) {
                const uint32_t kb = (uint32_t)__builtin_ctz(st);
                st &= st - 1u;
                queue[pos++] = (uint16_t)(l16 + kb);
            }
            const uint32_t total = (abl & 68u) ? 0u : lane_u32(incl, 63);
            MRG_PT(2);
            uint32_t nslow = 0;
            // an atomic LDS load (ds_read_b32): a volatile read of the same word compiled to a FLAT
            // load + s_waitcnt vmcnt(0), which made every tile wait for the previous tile's tail stores
            const bool may_claim =
                __builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
                (uint32_t)CAP;
            my_tokens += (abl & 4u) ? cnt : 0u;
            wave_sync_lds();

            // tokens of the queue, TWO per lane per round (entries q and q + 64: two independent LDS
            // dependency chains in one instruction stream, so each wait covers both)
            for (uint32_t base = 0; base < total; base += 128) {
                bool fa, sa, fb, sb;
                uint32_t sA, sB;
                uint64_t a0, a1, b0, b1;
                // both queue entries first, unconditionally (entries past `total` are stale but in
                // bounds), so the two chains share every LDS wait
                const uint32_t qa = base + (uint32_t)lane, qb = qa + 64u;
                const uint32_t ra = queue[min(qa, (uint32_t)QCAP - 1u)], rb = queue[min(qb, (uint32_t)QCAP - 1u)];
                uint32_t ga = extract(qa, ra, total, fa, sa, sA, a0, a1);
                uint32_t gb = extract(qb, rb, total, fb, sb, sB, b0, b1);
                if (!(abl & 1024u) && __any((ga | gb) != 0u)) {
                    squeeze(ga, a0, a1);
                    squeeze(gb, b0, b1);
                }
                // slow tokens (past the 2-segment window, or > 16 raw key bytes) are deferred: their
                // starts go to the consumed front of the queue (every lane has read both its entries,
                // and the deferred count never exceeds the entries read so far)
                const uint64_t ma = __ballot(sa), mb = __ballot(sb);
                if (ma | mb) {
                    const uint32_t ra = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
                    const uint32_t rb = __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
                    const uint32_t na = (uint32_t)__builtin_popcountll(ma);
                    if (sa) queue[nslow + ra] = (uint16_t)sA;
                    if (sb) queue[nslow + na + rb] = (uint16_t)sB;
                    nslow += na + (uint32_t)__builtin_popcountll(mb);
                }
                my_tokens += (fa ? 1u : 0u) + (fb ? 1u : 0u);
                const bool hv[2] = {fa, fb};
                const uint64_t kk0[2] = {a0, b0}, kk1[2] = {a1, b1};
                if constexpr (WIDE) {
                    wide_store(A, tails, fa, a0, a1);
                    wide_store(A, tails, fb, b0, b1);
                } else {
                    emit_fastN<2>(A, abl, hbits, table, tails, pool, pool16, hv, kk0, kk1, docid, may_claim);
                }
            }
            // deferred slow tokens, one per lane: through the tile's masks, or (a token running past
            // the first halo segment) the exact per-codepoint walker (forward reads only: the staged
            // bytes are [At, whi))
            MRG_PT(3);
            if (nslow && !(abl & 512u)) {
                wave_sync_lds();
                auto rd = [&](uint64_t a) -> uint32_t {
                    if (a >= At && a < whi) return (uint32_t)win[a - wbase];
                    return (uint32_t)gp(A.in)[a];
                };
                for (uint32_t base = 0; base < nslow; base += 64) {
                    const uint32_t q = base + (uint32_t)lane;
                    bool have = false;
                    uint64_t tk0 = 0, tk1 = 0, a = 0;
                    uint32_t tlen = 0, traw = 0;
                    if (q < nslow) {
                        const uint32_t s = queue[q];
                        a = At + s;
                        if (!(abl & 128u) && mask_walk(s, 64u, tk0, tk1, tlen, traw)) {
                            have = tlen > 0;
                        } else {
                            uint64_t e2;
                            if (walk_token(rd, a, doc_hi, A.counters, tk0, tk1, tlen, e2) && tlen > 0) {
                                have = true;
                                traw = (uint32_t)(e2 - a);
                            }
                        }
                    }
                    my_tokens += have ? 1u : 0u;
                    emit<CAP, IDX, WIDE>(A, table, tails, have, tk0, tk1, tlen, a, traw, docid);
                }
            }
        }
        MRG_PT(4);
    };

    // Main loop: two register sets, A and B.  Block c's loads were issued one block earlier; the
    // next block's loads go out before c is processed, so exactly five loads are younger than c's
    // when its data is first used.  Past the end, the "next" block is a reload of the current one.
    // the wave's pool state lives in LDS (s_pool[wv]): registers held across the main loop would add
    // to the kernel's SGPR spills; it is touched once per block
    constexpr uint64_t NONE = ~0ull;
    uint32_t dcur = 0;
    if (lane == 0) {
        s_pool[wv][0] = 0;
        s_pool[wv][1] = 0;
        s_pool[wv][2] = (blockIdx.x & 7u) | ((A.n_static < A.n_chunks ? 0u : 8u) << 8);
    }
    auto grab = [&]() -> uint64_t {
        uint32_t r = 0;
        if (lane == 0) r = atomicAdd(&s_next, 1u);
        const uint64_t c0 = wlo_b + (uint64_t)first_u32(r);
        if (c0 < whi_b) return c0;
        const uint64_t ns2 = A.n_static, np = A.n_chunks - ns2;   // (re-read: not held in registers)
        wave_sync_lds();
        const uint32_t cur = first_u32(s_pool[wv][0]), end = first_u32(s_pool[wv][1]);
        if (cur < end) {
            if (lane == 0) s_pool[wv][0] = cur + 1u;
            return ns2 + cur;
        }
        uint32_t pt = first_u32(s_pool[wv][2]);
        while ((pt >> 8) < 8u) {
            const uint32_t part = pt & 7u;
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(&s_stolen, (uint32_t)MRG_MAP_STEAL_K);
            if (first_u32(k) >= A.steal_max) {  // this workgroup's budget is spent
                pt = 8u << 8;
                break;
            }
            const uint32_t plo = (uint32_t)(np * part / 8u), phi = (uint32_t)(np * (part + 1u) / 8u);
            unsigned long long q = 0;
            if (lane == 0) q = atomicAdd(&A.pool_ctr[16u * part], (unsigned long long)MRG_MAP_STEAL_K);
            const uint32_t at = plo + first_u32((uint32_t)umin64(q, 0xFFFFFFFFull));
            if (at < phi) {
                if (lane == 0) {
                    s_pool[wv][0] = at + 1u;
                    s_pool[wv][1] = min(phi, at + (uint32_t)MRG_MAP_STEAL_K);
                    s_pool[wv][2] = pt;
                }
                // the document cursor walks forward (locate_blk); a search only when the chunk lies before
                // it (the wrap from part 7 to part 0)
                if (cp(A.chunk_base)[dcur] > ns2 + at) dcur = find_doc(A, ns2 + at);
                return ns2 + at;
            }
            pt = ((pt & 7u) + 1u) % 8u | (((pt >> 8) + 1u) << 8);
        }
        if (lane == 0) s_pool[wv][2] = pt;
        return NONE;
    };
    uint64_t c = grab();
    if (c != NONE) dcur = find_doc(A, c);
    Blk XA, XB;
    BlkInfo IA{}, IB{};
    // Make a block's registers available HERE (the compiler waits for its loads at this point, when
    // only older loads and stores are outstanding), before the next block's loads are issued --
    // otherwise the scheduler sinks the first use below them and the wait covers the new loads too.
    auto settle = [](Blk &X) {
        asm volatile("" : "+v"(X.v0.x), "+v"(X.v0.y), "+v"(X.v0.z), "+v"(X.v0.w), "+v"(X.v1.x), "+v"(X.v1.y),
                     "+v"(X.v1.z), "+v"(X.v1.w), "+v"(X.e.x), "+v"(X.e.y), "+v"(X.e.z), "+v"(X.e.w));
    };
    if (c != NONE) {
        IA = locate_blk(A, c, dcur);
#ifdef MRG_MAP_ABLATION
        first_blk = IA;
#endif
        load_blk(IA, XA);
        settle(XA);
    }
    while (c != NONE) {
        const uint64_t cB = grab();
        IB = cB != NONE ? locate_blk(A, cB, dcur) : IA;
        load_blk(IB, XB);
        process_blk(IA, XA, c, [&]() { settle(XB); });
        c = cB;
        if (c == NONE) break;
        const uint64_t cA = grab();
        IA = cA != NONE ? locate_blk(A, cA, dcur) : IB;
        load_blk(IA, XA);
        process_blk(IB, XB, c, [&]() { settle(XA); });
        c = cA;
    }
    MRG_PT(4);
#ifdef MRG_MAP_PROF
    __shared__ unsigned long long s_loop_end;
    if (tid == 0) s_loop_end = 0;
    lds_only_barrier();
    if (P && lane == 0) atomicMax(&s_loop_end, (unsigned long long)wall_clock64());
#endif
    // ---- non-ASCII tiles recorded by the main loop
    lds_only_barrier();   // s_ngen final
    if (s_ngen) __syncthreads();  // (uniform) the list is complete: its global writes, then the barrier
    {
        const uint32_t ng = s_ngen;
        for (uint32_t i = (uint32_t)wv; i < ng; i += NW) {
            {
                const uint32_t kk = first_u32(glist[i]);
                const uint64_t cb = kk / NSUB;
                uint32_t dgen = find_doc(A, cb);
                const BlkInfo b = locate_blk(A, cb, dgen);
                const TileInfo T = sub_tile(b, kk % NSUB);
                uint4 x0, x1;
                load(T, x0, x1);
                wave_sync_lds();
                if (j0 >= T.v0 && j0 < T.v1) reinterpret_cast<uint4 *>(win)[j0] = x0;
                if (has1 && j1 >= T.v0 && j1 < T.v1) reinterpret_cast<uint4 *>(win)[j1] = x1;
                wave_sync_lds();
                my_tokens += generic_tile<CAP, IDX, WIDE>(A, table, tails, win, T.At, T.t0, T.t1,
                                                    T.doc_lo, T.doc_hi, T.wlo, T.whi, T.docid);
            }
        }
    }

    MRG_PT(5);
    // ---- flush the LDS table into this workgroup's region, sorted by bucket (LDS-only barriers from
    // here on: the tail stores drain meanwhile; the kernel's end waits for them)
    lds_only_barrier();
    uint32_t my_tail = 0, my_tail16 = 0;
    if constexpr (WIDE) {  // the wide map: records per L1 bucket; a region past its capacity -> rerun
        uint32_t over = 0;
        for (uint32_t b = tid; b < A.wR * A.wB1r; b += WG) {
            const uint32_t n = s_wcur[b];
            gp(A.wcnt)[(uint64_t)b * gridDim.x + blockIdx.x] = n;
            my_tail += n;
            over += n > A.wcap ? n - A.wcap : 0u;
        }
        if (over) g_add(&A.counters[CNT_OVF], (unsigned long long)over);
    } else {
    uint16_t *s_rank = &s_q[0][0];
    GAS uint32_t *bcount = gp(A.bcount) + (uint64_t)blockIdx.x * MRG_NBUCKET;
    for (int b = tid; b < MRG_NBUCKET; b += WG) {  // appends made (may exceed the capacity)
        const uint32_t n = (uint32_t)(s_tcur[b] - (s_tend[b] - gp(A.bcap)[b]));
        my_tail += n;
        bcount[b] = n;
        if (!IDX) {
            const uint32_t n16 = (uint32_t)(s_tcur16[b] - (s_tend16[b] - gp(A.bcap16)[b]));
            my_tail += n16;
            my_tail16 += n16;
            gp(A.bcount16)[(uint64_t)blockIdx.x * MRG_NBUCKET + b] = n16;
        }
    }
    for (int b = tid; b <= MRG_NBUCKET; b += WG) s_hist[b] = 0;
    lds_only_barrier();
    MRG_FT(0);
    for (int i = tid; i < CAP; i += WG) {
        const KeyPair k = s_key[i];
        if (k.a == MRG_EMPTY_K0) continue;
        const uint32_t b = bucket_of(key_hash(k.a, k.b, IDX ? s_doc[i] : MRG_EMPTY_DOC, A.hash_bits));
        s_rank[i] = (uint16_t)atomicAdd(&s_hist[b], 1u);
    }
    lds_only_barrier();
    MRG_FT(1);
    if (tid < 64) {  // exclusive scan of the bucket histogram by one wave
        uint32_t run = 0;
        for (int b0 = 0; b0 < MRG_NBUCKET; b0 += 64) {
            const uint32_t v = s_hist[b0 + lane];
            const uint32_t inc = wave_incl_scan(v);
            s_hist[b0 + lane] = run + inc - v;
            run += lane_u32(inc, 63);
        }
        if (lane == 0) s_hist[MRG_NBUCKET] = run;
    }
    lds_only_barrier();
    MRG_FT(2);
    GAS uint32_t *foff = gp(A.foff) + (uint64_t)blockIdx.x * (MRG_NBUCKET + 1);
    for (int b = tid; b <= MRG_NBUCKET; b += WG) foff[b] = s_hist[b];
    const uint64_t reg = (uint64_t)blockIdx.x * CAP;
    for (int i = tid; i < CAP; i += WG) {
        const KeyPair k = s_key[i];
        if (k.a == MRG_EMPTY_K0) continue;
        const uint32_t d = IDX ? s_doc[i] : MRG_EMPTY_DOC;
        const uint32_t b = bucket_of(key_hash(k.a, k.b, d, A.hash_bits));
        const uint64_t pos2 = reg + s_hist[b] + s_rank[i];
        gp(A.fk0)[pos2] = k.a;
        gp(A.fk1)[pos2] = k.b;
        gp(A.fcnt)[pos2] = s_cnt[i];
        if (IDX) gp(A.fdoc)[pos2] = d;
    }
    }
    MRG_FT(3);
    // token and tail totals: waves -> LDS -> one device atomic per workgroup and counter (a wave
    // atomic each put 8 K atomics on two counters at the very end of the launch)
    uint32_t t = my_tokens, ttl = my_tail, t16 = my_tail16;
    for (int off = 32; off > 0; off >>= 1) {
        t += __shfl_down(t, off);
        ttl += __shfl_down(ttl, off);
        t16 += __shfl_down(t16, off);
    }
    if (lane == 0) {
        atomicAdd(&s_tot[0], t);
        atomicAdd(&s_tot[1], ttl);
        if (t16) atomicAdd(&s_tot[2], t16);
    }
    lds_only_barrier();
    if (tid == 0) {
        g_add(&A.counters[CNT_TOKENS], (unsigned long long)s_tot[0]);
        g_add(&A.counters[CNT_REC], (unsigned long long)s_tot[1]);
        if (s_tot[2]) g_add(&A.counters[CNT_REC16], (unsigned long long)s_tot[2]);
        if (s_ngen + s_nuni) g_add(&A.counters[CNT_NONASCII], (unsigned long long)(s_ngen + s_nuni));
        gp(A.lcount)[blockIdx.x] = s_lcnt;
        if (s_lcnt) g_add(&A.counters[CNT_LONG], (unsigned long long)s_lcnt);
    }
    MRG_FT(4);
    MRG_PT(6);
#ifdef MRG_MAP_PROF
    if (P && lane == 0) {
        for (int i = 0; i < 7; ++i) g_add(&A.prof[i], (unsigned long long)pacc[i]);
    }
    if (P && tid == 0) {
        gp(A.prof)[8 + 8 * blockIdx.x] = wg_t0;
        gp(A.prof)[9 + 8 * blockIdx.x] = wall_clock64();
        gp(A.prof)[10 + 8 * blockIdx.x] = s_loop_end;   // the last wave's main-loop end
        for (int i = 0; i < 5; ++i) gp(A.prof)[11 + 8 * blockIdx.x + i] = ftv[i];   // the flush's steps
    }
#endif
}

// Long tokens: filter the raw token bytes (drop X codepoints), fingerprint (FNV-1a-64 of the key
// bytes; internal grouping only), packed prefix and key length.  Input was validated by k_map.
__global__ void k_long_prep(const uint8_t *in, const uint64_t *lstart, const uint32_t *llen, uint64_t n,
                            uint64_t *ok0, uint64_t *ok1, uint32_t *oflen, uint64_t *oflen64, uint64_t *ofp,
                            uint32_t hash_bits, int verbatim) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = lstart[i], e = a + llen[i];
    auto rd = [&](uint64_t x) -> uint32_t { return in[x]; };
    uint64_t k0 = 0, k1 = 0, h = 0xcbf29ce484222325ull;
    uint32_t L = 0;
    for (uint64_t p = a; p < e;) {
        if (verbatim) {  // the range already holds exactly the key bytes (exchange heap, text key)
            const uint32_t by = in[p++];
            mrg_key_append(k0, k1, L, by);
            h = (h ^ by) * 0x100000001b3ull;
            ++L;
            continue;
        }
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
                              const uint64_t *dst_off, uint8_t *heap, int verbatim) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a = lstart[i], e = a + llen[i];
    auto rd = [&](uint64_t x) -> uint32_t { return in[x]; };
    uint8_t *dst = heap + dst_off[i];
    if (verbatim) {
        for (uint64_t p = a; p < e; ++p) *dst++ = in[p];
        return;
    }
    for (uint64_t p = a; p < e;) {
        uint32_t cp, raw;
        int l = mrg_utf8_decode(rd, p, e, &cp, &raw);
        if (!l) l = 1;
        if (mrg_uclass(cp) == MRG_CLS_W)
            for (int b = 0; b < l; ++b) *dst++ = (uint8_t)(raw >> (8 * b));
        p += (uint64_t)l;
    }
}

// Dense long-token records (see mrg_launch_long_compact): block w < grid copies region w, block grid
// the shared list; each block finds its output offset by summing the regions before it.
__global__ void k_long_compact(const uint64_t *__restrict__ rs, const uint32_t *__restrict__ rl,
                               const uint32_t *__restrict__ rd, const uint32_t *__restrict__ lcount, uint32_t lper,
                               uint64_t lovf, const unsigned long long *__restrict__ counters, uint32_t grid,
                               uint64_t *__restrict__ start, uint32_t *__restrict__ len, uint32_t *__restrict__ doc) {
    __shared__ unsigned long long s_off;
    const uint32_t w = blockIdx.x;
    if (threadIdx.x == 0) s_off = 0;
    __syncthreads();
    unsigned long long part = 0;
    for (uint32_t v = threadIdx.x; v < w; v += blockDim.x) part += min(lcount[v], lper);
    if (part) atomicAdd(&s_off, part);
    __syncthreads();
    const uint64_t off = s_off;
    const uint64_t n = w < grid ? (uint64_t)min(lcount[w], lper) : umin64(counters[CNT_LONGX], lovf);
    const uint64_t src = (uint64_t)w * lper;  // block grid: the list right after the regions
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
        start[off + i] = rs[src + i];
        len[off + i] = rl[src + i];
        doc[off + i] = rd[src + i];
    }
}

}  // namespace

void mrg_launch_long_compact(const MapArgs &A, int grid, uint64_t *start, uint32_t *len, uint32_t *doc,
                             hipStream_t s) {
    hipLaunchKernelGGL(k_long_compact, dim3((unsigned)grid + 1), dim3(256), 0, s, A.lstart, A.llen, A.ldoc, A.lcount,
                       A.lper, A.lovf, A.counters, (uint32_t)grid, start, len, doc);
}

template <int CAP, bool IDX, bool WIDE = false>
static void launch_map_t(const MapArgs *a, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_map<CAP, IDX, WIDE>), dim3(grid), dim3(WG), 0, s, a);
}

static int map_cap_for(int app, int lds_cap) {
    (void)app;
    return lds_cap >= 4096 ? 4096 : 2048;
}

void mrg_launch_map(const MapArgs *h, MapArgs *a, int app, int grid, int lds_cap, hipStream_t s, bool wide) {
    const bool idx = app == 1;
    if (h) (void)hipMemcpyAsync(a, h, sizeof(MapArgs), hipMemcpyHostToDevice, s);
    if (wide && !idx) {  // the wide map (no LDS table): one layout whatever lds_cap
        launch_map_t<2048, false, true>(a, grid, s);
        return;
    }
    if (map_cap_for(app, lds_cap) == 4096) {
        if (idx) launch_map_t<4096, true>(a, grid, s);
        else launch_map_t<4096, false>(a, grid, s);
    } else {
        if (idx) launch_map_t<2048, true>(a, grid, s);
        else launch_map_t<2048, false>(a, grid, s);
    }
}

int mrg_map_cap(int app, int lds_cap) { return map_cap_for(app, lds_cap); }

// BLK-byte blocks of a document [lo, hi): on the 16-byte grid starting at lo & ~15
uint64_t mrg_map_tiles(uint64_t lo, uint64_t hi) {
    if (hi <= lo) return 0;
    return (hi - (lo & ~15ull) + BLK - 1) / BLK;
}

int mrg_map_max_grid(int app, int lds_cap, int device) {
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
    int per = 1;
    hipError_t e;
    if (map_cap_for(app, lds_cap) == 4096)
        e = app == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<4096, true, false>, WG, 0)
                     : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<4096, false, false>, WG, 0);
    else if (app == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<2048, true, false>, WG, 0);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_map<2048, false, false>, WG, 0);
    if (e != hipSuccess || per < 1) per = 1;
    return ncu * per;
}

void mrg_launch_long_prep(const uint8_t *base, const uint64_t *start, const uint32_t *rawlen, uint64_t n,
                          uint64_t *k0, uint64_t *k1, uint32_t *flen, uint64_t *flen64, uint64_t *fp,
                          uint32_t hash_bits, int verbatim, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_long_prep, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, base, start, rawlen, n, k0,
                       k1, flen, flen64, fp, hash_bits, verbatim);
}

void mrg_launch_long_gather(const uint8_t *base, const uint64_t *start, const uint32_t *rawlen, uint64_t n,
                            const uint64_t *dst_off, uint8_t *heap, int verbatim, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_long_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, base, start, rawlen, n,
                       dst_off, heap, verbatim);
}
