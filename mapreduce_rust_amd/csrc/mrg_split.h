// mrg_split.h -- key order, splitter search and the partition function shared by the wide
// aggregation (k_wide.hip) and the wide map (k_map.hip).  Device code only.
//
// Keys are compared as (k0, k1) unsigned = their bytes (mrg_device.h packing); the partition of a key
// is SipHash-1-3(key bytes ++ 0xFF) % R, src/mr/worker.rs:111-115, 129.
#pragma once
#include "mrg_device.h"

__device__ __forceinline__ bool key_lt(uint64_t a0, uint64_t a1, uint64_t b0, uint64_t b1) {
    return a0 < b0 || (a0 == b0 && a1 < b1);
}

// The 64 key bits from bit h on (bit 0 = the most significant bit of k0), zero past bit 127.
__device__ __forceinline__ uint64_t key_bits_from(uint64_t k0, uint64_t k1, uint32_t h) {
    return h == 0 ? k0 : (h < 64 ? (k0 << h) | (k1 >> (64 - h)) : k1 << (h - 64));
}
// leading bits two keys share (128 if equal)
__device__ __forceinline__ uint32_t common_bits(uint64_t a0, uint64_t a1, uint64_t b0, uint64_t b1) {
    const uint64_t x0 = a0 ^ b0, x1 = a1 ^ b1;
    return x0 ? (uint32_t)__builtin_clzll(x0) : (x1 ? 64u + (uint32_t)__builtin_clzll(x1) : 128u);
}

// Splitter index: m sorted splitters share their top cp bits; the next IB bits of a key select
// ix[v] .. ix[v + 1], the splitters carrying those same bits, so a lookup compares the key with
// that handful (usually 0-2) instead of walking log2(m) levels of 16-byte LDS reads.  A key whose
// top cp bits differ from the splitters' lies below all of them or above all of them.
template <uint32_t IB, class IX>
struct SplitIndex {
    const uint64_t *spl;  // m (k0, k1) pairs in LDS
    const IX *ix;         // [2^IB + 1] in LDS
    uint32_t m, cp;
    __device__ __forceinline__ static uint32_t slot(uint64_t k0, uint64_t k1, uint32_t cp) {
        return (uint32_t)(key_bits_from(k0, k1, cp) >> (64 - IB));
    }
    __device__ __forceinline__ static uint32_t prefix_bits(const uint64_t *spl, uint32_t m) {
        return min(common_bits(spl[0], spl[1], spl[2 * (m - 1)], spl[2 * (m - 1) + 1]), 128u - IB);
    }
    // the index of m >= 1 splitters, by threads tid, tid + nt, ... (the caller synchronises)
    __device__ __forceinline__ static void build(const uint64_t *spl, uint32_t m, IX *ix, uint32_t tid, uint32_t nt) {
        const uint32_t cp = prefix_bits(spl, m);
        for (uint32_t v = tid; v <= (1u << IB); v += nt) {  // first splitter whose slot is >= v
            uint32_t lo = 0, hi = m;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (slot(spl[2 * mid], spl[2 * mid + 1], cp) < v) lo = mid + 1;
                else hi = mid;
            }
            ix[v] = (IX)lo;
        }
    }
    // number of splitters <= key (m >= 1)
    __device__ __forceinline__ uint32_t upper(uint64_t k0, uint64_t k1) const {
        const uint64_t p0 = spl[0], p1 = spl[1];
        if (common_bits(k0, k1, p0, p1) < cp) return key_lt(k0, k1, p0, p1) ? 0u : m;
        const uint32_t v = slot(k0, k1, cp);
        uint32_t lo = ix[v], hi = ix[v + 1];
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (key_lt(k0, k1, spl[2 * mid], spl[2 * mid + 1])) hi = mid;
            else lo = mid + 1;
        }
        return lo;
    }
};
typedef SplitIndex<12, uint16_t> LeafIndex;   // L2: <= 1023 leaf splitters per L1 bucket
typedef SplitIndex<8, uint8_t> L1Index;       // L1: <= 63 splitters per partition

__device__ __forceinline__ uint32_t part_of(uint64_t k0, uint64_t k1, uint32_t R) {
    const uint64_t h = mrg_siphash_short(k0, k1, mrg_short_len(k0, k1));
    if ((R & (R - 1u)) == 0u) return (uint32_t)h & (R - 1u);   // uniform: no 64-bit division
    return (uint32_t)(h % (uint64_t)R);
}
