// k_map.hip -- the map kernel: tokenize + local combine (MI355X / gfx950).
//
// Replaces wc::map (src/app/wc.rs:6-13) -- delete every codepoint outside \w ∪ \s, split on
// White_Space -- fused with the per-token part of write_key_value_to_file (src/mr/worker.rs:127-131).
// The partition index (worker.rs:129) is computed later, once per DISTINCT key (k_keys.hip), since
// SipHash(key) % R is a pure function of the key.  Also validates UTF-8 like read_to_string
// (worker.rs:75): the first invalid byte offset is reported, the job fails with MRG_EUTF8.
//
// Layout: documents back to back in one HBM buffer; each document is cut into 4 KiB tiles; a
// persistent grid of 256-thread workgroups walks the tiles.  Per tile the workgroup stages
// [tile - 16 B, tile + 4 KiB + 256 B) into LDS with 16-byte loads (coalesced), then every lane owns a
// 16-byte segment: tokens whose first codepoint starts in the segment are the lane's; a lane walks
// its tokens (continuing past the segment end through LDS, or HBM beyond the halo) and packs the
// first 16 key bytes big-endian into (k0, k1).
// Keys of <= 16 bytes are inserted into a workgroup-private LDS hash table (exact: the packed key
// IS the identity, no fingerprint); count += 1.  Insert misses (table region full) become records
// in HBM.  Keys > 16 bytes become long-token records (start, raw length, doc) resolved by the
// collision-safe fingerprint sort (k_keys.hip).  At the end every LDS table is flushed as records.
#include "mrg_device.h"
#include "mrg_internal.h"

namespace {

constexpr int WG = MRG_MAP_WG;
constexpr int SEG = MRG_MAP_SEG;
constexpr int TILE = MRG_MAP_TILE;
constexpr int HALO = MRG_MAP_HALO;
constexpr int BEHIND = MRG_MAP_BEHIND;
constexpr int TILE_LDS = BEHIND + TILE + HALO + 32;   // staged window incl. 16-B alignment slack
constexpr int MAX_PROBE = 8;

struct Window {
    const uint8_t *lds;
    const uint8_t *g;
    uint64_t lo, hi, wbase;
    __device__ __forceinline__ uint32_t operator()(uint64_t a) const {
        return (a >= lo && a < hi) ? (uint32_t)lds[a - wbase] : (uint32_t)g[a];
    }
};

__device__ __forceinline__ void report_error(unsigned long long *counters, uint64_t pos) {
    atomicMin(&counters[CNT_ERRPOS], (unsigned long long)pos);
}

// Workgroup LDS table, open addressing with a monotone claim protocol:
// a slot goes EMPTY -> k0 set -> k1 set (-> doc set) and never back; a key may complete a slot
// whose already-set words equal its own.  Two lanes racing on one slot therefore agree on its
// owner, and every key lives in exactly one slot without locks.
template <int CAP, bool IDX>
struct LdsTable {
    unsigned long long *k0, *k1;
    unsigned int *cnt, *doc;

    __device__ __forceinline__ bool insert(uint64_t a, uint64_t b, uint32_t d, uint32_t hash_bits) {
        uint64_t h = mrg_key_mix(a, b, d);
        if (hash_bits) h &= (1ull << hash_bits) - 1u;
        uint32_t slot = (uint32_t)(h ^ (h >> 29)) & (CAP - 1);
        for (int p = 0; p < MAX_PROBE; ++p) {
            const unsigned long long x = atomicCAS(&k0[slot], MRG_EMPTY_K0, (unsigned long long)a);
            if (x == MRG_EMPTY_K0 || x == a) {
                const unsigned long long y = atomicCAS(&k1[slot], MRG_EMPTY_K1, (unsigned long long)b);
                if (y == MRG_EMPTY_K1 || y == b) {
                    bool ok = true;
                    if (IDX) {
                        const unsigned int z = atomicCAS(&doc[slot], MRG_EMPTY_DOC, d);
                        ok = (z == MRG_EMPTY_DOC || z == d);
                    }
                    if (ok) {
                        atomicAdd(&cnt[slot], 1u);
                        return true;
                    }
                }
            }
            slot = (slot + 1u) & (CAP - 1);
        }
        return false;
    }
};

template <int CAP, bool IDX>
__global__ __launch_bounds__(WG) void k_map(MapArgs A) {
    __shared__ __attribute__((aligned(16))) uint8_t s_tile[TILE_LDS];
    __shared__ unsigned long long s_k0[CAP];
    __shared__ unsigned long long s_k1[CAP];
    __shared__ unsigned int s_cnt[CAP];
    __shared__ unsigned int s_doc[IDX ? CAP : 1];

    const int tid = threadIdx.x;
    for (int i = tid; i < CAP; i += WG) {
        s_k0[i] = MRG_EMPTY_K0;
        s_k1[i] = MRG_EMPTY_K1;
        s_cnt[i] = 0;
        if (IDX) s_doc[i] = MRG_EMPTY_DOC;
    }
    LdsTable<CAP, IDX> table{s_k0, s_k1, s_cnt, s_doc};
    uint64_t my_tokens = 0;

    for (uint64_t c = blockIdx.x; c < A.n_chunks; c += gridDim.x) {
        // ---- locate the tile (uniform across the workgroup)
        uint32_t lo_d = 0, hi_d = A.n_docs;  // chunk_base[d] <= c < chunk_base[d+1]
        while (hi_d - lo_d > 1) {
            const uint32_t mid = (lo_d + hi_d) >> 1;
            if (A.chunk_base[mid] <= c) lo_d = mid; else hi_d = mid;
        }
        const uint32_t d = lo_d;
        const uint64_t doc_lo = A.doc_off[d], doc_hi = A.doc_off[d + 1];
        const uint64_t t0 = doc_lo + (c - A.chunk_base[d]) * (uint64_t)TILE;
        const uint64_t t1 = min(t0 + (uint64_t)TILE, doc_hi);
        const uint32_t docid = A.doc_id ? A.doc_id[d] : d;

        Window W;
        W.lds = s_tile;
        W.g = A.in;
        W.lo = t0 - min((uint64_t)BEHIND, t0 - doc_lo);
        W.hi = min(t1 + (uint64_t)HALO, doc_hi);
        W.wbase = W.lo & ~15ull;
        const uint32_t nvec = (uint32_t)((((W.hi + 15u) & ~15ull) - W.wbase) >> 4);

        __syncthreads();  // previous tile fully consumed
        for (uint32_t v = tid; v < nvec; v += WG)
            reinterpret_cast<uint4 *>(s_tile)[v] = reinterpret_cast<const uint4 *>(A.in + W.wbase)[v];
        __syncthreads();

        // ---- lane segment
        const uint64_t s0 = t0 + (uint64_t)tid * SEG;
        const uint64_t s1 = min(s0 + (uint64_t)SEG, t1);
        bool done = s0 >= t1;
        uint64_t p = s0;
        bool prevS = true;
        if (!done && s0 > doc_lo) {
            // skip continuation bytes: they belong to a codepoint that starts before s0
            uint32_t j = 0;
            while (s0 + j < s1 && mrg_is_cont(W(s0 + j))) ++j;
            p = s0 + j;
            // find the lead of the codepoint ending at p - 1 (at most 3 continuation bytes back)
            uint32_t k = 1;
            while (k <= 3 && p - k >= doc_lo && mrg_is_cont(W(p - k))) ++k;
            const uint64_t q = p - k;
            if (q < doc_lo || mrg_is_cont(W(q))) {
                report_error(A.counters, s0);   // orphan continuation bytes
                done = true;
            } else {
                uint32_t cp, raw;
                const int l = mrg_utf8_decode(W, q, doc_hi, &cp, &raw);
                if (j > 0 && (l == 0 || q + (uint64_t)l != p)) {
                    report_error(A.counters, s0);   // continuation bytes not covered by their lead
                    done = true;
                }
                // an invalid lead itself is reported by the lane that owns it
                prevS = (l > 0 && q + (uint64_t)l == p) ? (mrg_uclass(cp) == MRG_CLS_S) : false;
            }
            if (p >= s1) done = true;
        }

        // ---- token rounds: every lane produces at most one token per round, then the wave
        //      inserts all of them together (full-wave LDS atomics instead of 1-lane divergence)
        for (;;) {
            bool have = false;
            uint64_t tk0 = 0, tk1 = 0, tstart = 0;
            uint32_t tlen = 0, traw = 0;
            while (!done) {
                if (p >= s1) { done = true; break; }
                uint32_t cp, raw;
                int l = mrg_utf8_decode(W, p, doc_hi, &cp, &raw);
                if (!l) { report_error(A.counters, p); done = true; break; }
                uint32_t c = mrg_uclass(cp);
                if (c == MRG_CLS_S) { prevS = true; p += (uint64_t)l; continue; }
                if (!prevS) { p += (uint64_t)l; continue; }
                // token starts at p: walk to the next White_Space codepoint or the document end
                const uint64_t start = p;
                uint64_t a0 = 0, a1 = 0;
                uint32_t L = 0;
                for (;;) {
                    if (c == MRG_CLS_W) {
                        for (int b = 0; b < l; ++b) {
                            mrg_key_append(a0, a1, L, (raw >> (8 * b)) & 0xFFu);
                            ++L;
                        }
                    }
                    p += (uint64_t)l;
                    if (p >= doc_hi) break;
                    l = mrg_utf8_decode(W, p, doc_hi, &cp, &raw);
                    if (!l) { report_error(A.counters, p); done = true; break; }
                    c = mrg_uclass(cp);
                    if (c == MRG_CLS_S) break;
                }
                prevS = false;
                if (L > 0 && !done) {
                    have = true;
                    tk0 = a0; tk1 = a1; tlen = L; tstart = start; traw = (uint32_t)(p - start);
                    break;
                }
            }
            if (!__any(have)) break;
            my_tokens += have ? 1u : 0u;
            const bool is_long = have && tlen > 16u;
            bool tail = false;
            if (have && !is_long) tail = !table.insert(tk0, tk1, IDX ? docid : MRG_EMPTY_DOC, A.hash_bits);
            const uint64_t ri = mrg_wave_append(&A.counters[CNT_REC], tail);
            if (tail && ri < A.rcap) {
                A.rk0[ri] = tk0; A.rk1[ri] = tk1; A.rcnt[ri] = 1u;
                if (IDX) A.rdoc[ri] = docid;
            }
            const uint64_t li = mrg_wave_append(&A.counters[CNT_LONG], is_long);
            if (is_long && li < A.lcap) {
                A.lstart[li] = tstart; A.llen[li] = traw; A.ldoc[li] = docid;
            }
        }
    }

    // ---- flush the LDS table as records
    __syncthreads();
    for (int i0 = 0; i0 < CAP; i0 += WG) {
        const int i = i0 + tid;
        const bool full = s_k0[i] != MRG_EMPTY_K0;
        const uint64_t ri = mrg_wave_append(&A.counters[CNT_REC], full);
        if (full && ri < A.rcap) {
            A.rk0[ri] = s_k0[i]; A.rk1[ri] = s_k1[i]; A.rcnt[ri] = s_cnt[i];
            if (IDX) A.rdoc[ri] = s_doc[i];
        }
    }
    // token count
    uint64_t t = my_tokens;
    for (int off = 32; off > 0; off >>= 1) t += __shfl_down(t, off);
    if (mrg_lane() == 0) atomicAdd(&A.counters[CNT_TOKENS], (unsigned long long)t);
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
static void launch_map_t(const MapArgs &a, int grid, hipStream_t s) {
    hipLaunchKernelGGL((k_map<CAP, IDX>), dim3(grid), dim3(WG), 0, s, a);
}

void mrg_launch_map(const MapArgs &a, int app, int grid, int lds_cap, hipStream_t s) {
    const bool idx = app == 1;
    if (lds_cap >= 4096) { if (idx) launch_map_t<4096, true>(a, grid, s); else launch_map_t<4096, false>(a, grid, s); }
    else if (lds_cap >= 2048) { if (idx) launch_map_t<2048, true>(a, grid, s); else launch_map_t<2048, false>(a, grid, s); }
    else { if (idx) launch_map_t<1024, true>(a, grid, s); else launch_map_t<1024, false>(a, grid, s); }
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

void mrg_launch_long_gather(const uint8_t *in, const uint64_t *lstart, const uint32_t *llen, uint64_t n,
                            const uint64_t *dst_off, uint8_t *heap, hipStream_t s) {
    if (!n) return;
    hipLaunchKernelGGL(k_long_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, lstart, llen, n,
                       dst_off, heap);
}
