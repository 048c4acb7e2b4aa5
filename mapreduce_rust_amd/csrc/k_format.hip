// k_format.hip -- reduce-side grouping and the mr-{r}.txt writer (gfx950).
//
// Restates the reduce loop of Worker::reduce (src/mr/worker.rs:165-184) over keys that are already
// distinct and sorted by (partition, key bytes): each key is one group; the line is
// format!("{} {}\n", key, reduce(key, values)) (worker.rs:179) with wc::reduce = values.len()
// (src/app/wc.rs:15-17).  The reference never writes the LAST group of a partition (the loop ends
// without a final flush), so with drop_last the largest key of every partition is omitted.
// Indexer (build-defined): keys are (word, doc) pairs sorted by (partition, word, doc name); one line
// per word: "{word} {n} {doc1,doc2,...}".
// Lengths -> exclusive scan -> every line written at its offset; partitions are contiguous.
#include <algorithm>

#include "mrg_device.h"
#include "mrg_internal.h"

namespace {

inline dim3 grid_for(uint64_t n, int b = 256) { return dim3((unsigned)((n + b - 1) / b)); }

__device__ __forceinline__ uint32_t key_byte_at(const KeySet &ks, const uint8_t *heap, uint32_t e, uint32_t i,
                                                uint64_t k0, uint64_t k1) {
    return ks.len[e] > 16u ? heap[ks.hoff[e] + i] : mrg_key_byte(k0, k1, i);
}

// full-key order of two sorted records with equal (part, k0, k1): bytes beyond 16, then length
__device__ int cmp_full(const SortRec &a, const SortRec &b, const KeySet &ks, const uint8_t *heap) {
    const uint32_t la = ks.len[a.idx], lb = ks.len[b.idx];
    const uint32_t l = la < lb ? la : lb;
    for (uint32_t i = 16; i < l; ++i) {
        const uint32_t x = heap[ks.hoff[a.idx] + i], y = heap[ks.hoff[b.idx] + i];
        if (x != y) return x < y ? -1 : 1;
    }
    if (la != lb) return la < lb ? -1 : 1;
    return a.doc < b.doc ? -1 : (a.doc > b.doc ? 1 : 0);
}

__device__ __forceinline__ bool same_prefix(const SortRec &a, const SortRec &b) {
    return a.part == b.part && a.k0 == b.k0 && a.k1 == b.k1;
}

// runs of equal (part, 16-byte prefix) that involve a long key: insertion sort by full bytes
__global__ void k_fix_runs(SortRec *r, uint64_t n, KeySet ks, const uint8_t *heap) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i > 0 && same_prefix(r[i - 1], r[i])) return;          // not a run head
    uint64_t e = i + 1;
    bool any_long = ks.len[r[i].idx] > 16u;
    while (e < n && same_prefix(r[i], r[e])) {
        any_long |= ks.len[r[e].idx] > 16u;
        ++e;
    }
    if (e - i < 2 || !any_long) return;
    for (uint64_t a = i + 1; a < e; ++a) {
        const SortRec x = r[a];
        uint64_t b = a;
        while (b > i && cmp_full(x, r[b - 1], ks, heap) < 0) {
            r[b] = r[b - 1];
            --b;
        }
        r[b] = x;
    }
}

// ---------------------------------------------------------------- wc
// a record's key length and count: from the record itself when carried (mrg_launch_make_sortrec),
// else gathered from the key set
__device__ __forceinline__ void len_cnt(const SortRec &r, const KeySet &ks, int carried, uint32_t &len, uint64_t &c) {
    if (carried) {
        c = (uint64_t)r.doc | ((uint64_t)(r.pad >> 8) << 32);
        len = r.pad & 0xFFu;
        if (len > 16u) len = ks.len[r.idx];
    } else {
        len = ks.len[r.idx];
        c = ks.cnt[r.idx];
    }
}

__global__ void k_wc_len(const SortRec *r, uint64_t n, KeySet ks, int drop_last, int carried, uint64_t *L) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const SortRec x = r[i];
    const bool last = (i + 1 == n) || r[i + 1].part != x.part;
    uint32_t len;
    uint64_t c;
    len_cnt(x, ks, carried, len, c);
    L[i] = (drop_last && last) ? 0ull : (uint64_t)len + 2u + mrg_ndigits(c);
}

__device__ __forceinline__ uint8_t *put_u64(uint8_t *o, uint64_t v, uint32_t nd) {
    if (v <= 0xFFFFFFFFull) {  // 32-bit division (a 64-bit one is a long software sequence)
        uint32_t w = (uint32_t)v;
        for (uint32_t k = nd; k > 0; --k) {
            o[k - 1] = (uint8_t)('0' + w % 10u);
            w /= 10u;
        }
        return o + nd;
    }
    for (uint32_t k = nd; k > 0; --k) {
        o[k - 1] = (uint8_t)('0' + v % 10u);
        v /= 10u;
    }
    return o + nd;
}

__global__ void k_wc_write(const SortRec *r, uint64_t n, KeySet ks, const uint8_t *heap, const uint64_t *L,
                           const uint64_t *O, int carried, uint8_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || L[i] == 0) return;
    const SortRec x = r[i];  // read once: the byte stores below may alias any global pointer
    const uint32_t e = x.idx;
    uint32_t len;
    uint64_t c;
    len_cnt(x, ks, carried, len, c);
    uint8_t *o = out + O[i];
    if (len <= 16u) {
        const uint64_t k0 = x.k0, k1 = x.k1;
        for (uint32_t b = 0; b < len; ++b) o[b] = (uint8_t)mrg_key_byte(k0, k1, b);
    } else {
        const uint8_t *src = heap + ks.hoff[e];
        for (uint32_t b = 0; b < len; ++b) o[b] = src[b];
    }
    o += len;
    *o++ = ' ';
    o = put_u64(o, c, mrg_ndigits(c));
    *o = '\n';
}

// part_off[p] = byte offset of the first element with part >= p  (elements: lines or groups)
__global__ void k_part_off(const SortRec *r, const uint64_t *pos, uint64_t n, uint32_t R, const uint64_t *gidx,
                           const uint64_t *total_p, uint64_t *part_off) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    // element i is the first of its partition run; previous partition id (or -1)
    const int64_t prev = i == 0 ? -1 : (int64_t)r[gidx ? gidx[i - 1] : i - 1].part;
    const int64_t cur = i == n ? (int64_t)R : (int64_t)r[gidx ? gidx[i] : i].part;
    if (cur == prev) return;
    const uint64_t off = i == n ? *total_p : pos[i];
    for (int64_t p = prev + 1; p <= cur; ++p) part_off[p] = off;
}

__global__ void k_total(const uint64_t *L, const uint64_t *O, uint64_t n, uint64_t *total) {
    *total = n ? O[n - 1] + L[n - 1] : 0ull;
}

// ---------------------------------------------------------------- indexer
__device__ bool same_key(const SortRec &a, const SortRec &b, const KeySet &ks, const uint8_t *heap) {
    if (!same_prefix(a, b)) return false;
    const uint32_t la = ks.len[a.idx], lb = ks.len[b.idx];
    if (la != lb) return false;
    for (uint32_t i = 16; i < la; ++i)
        if (heap[ks.hoff[a.idx] + i] != heap[ks.hoff[b.idx] + i]) return false;
    return true;
}

__global__ void k_idx_heads(const SortRec *r, uint64_t n, KeySet ks, const uint8_t *heap,
                            const uint64_t *name_off, uint64_t *head, uint64_t *nl) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    head[i] = (i == 0 || !same_key(r[i - 1], r[i], ks, heap)) ? 1u : 0u;
    const uint32_t d = r[i].doc;  // doc rank
    nl[i] = name_off[d + 1] - name_off[d] + 1u;   // name + ',' or '\n'
}

__global__ void k_idx_groups(const uint64_t *head, const uint64_t *E, uint64_t n, uint64_t *H) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && head[i]) H[E[i]] = i;
}

__global__ void k_idx_glen(const SortRec *r, uint64_t n, uint64_t G, KeySet ks, const uint64_t *H,
                           const uint64_t *P, uint64_t Ptotal, int drop_last, uint64_t *GL) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G) return;
    const uint64_t s = H[g], e = g + 1 < G ? H[g + 1] : n;
    const bool last = (g + 1 == G) || r[H[g + 1]].part != r[s].part;
    if (drop_last && last) { GL[g] = 0; return; }
    const uint64_t size = e - s;
    const uint64_t names = (e < n ? P[e] : Ptotal) - P[s];
    GL[g] = (uint64_t)ks.len[r[s].idx] + 1u + mrg_ndigits(size) + 1u + names;
}

__global__ void k_idx_write(const SortRec *r, uint64_t n, uint64_t G, KeySet ks, const uint8_t *heap,
                            const uint64_t *head, const uint64_t *E, const uint64_t *H, const uint64_t *P,
                            const uint64_t *GL, const uint64_t *GO, const uint8_t *names, const uint64_t *name_off,
                            uint8_t *out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t g = E[i] + head[i] - 1u;
    if (GL[g] == 0) return;
    const uint64_t s = H[g], e = g + 1 < G ? H[g + 1] : n;
    const uint64_t size = e - s;
    const uint32_t nd = mrg_ndigits(size);
    const uint32_t es = r[s].idx;
    const uint32_t klen = ks.len[es];
    uint8_t *o = out + GO[g];
    if (i == s) {
        for (uint32_t b = 0; b < klen; ++b) o[b] = (uint8_t)key_byte_at(ks, heap, es, b, r[s].k0, r[s].k1);
        o[klen] = ' ';
        put_u64(o + klen + 1, size, nd);
        o[klen + 1 + nd] = ' ';
    }
    uint8_t *q = o + klen + 1 + nd + 1 + (P[i] - P[s]);
    const uint32_t d = r[i].doc;
    const uint64_t a = name_off[d], z = name_off[d + 1];
    for (uint64_t k = a; k < z; ++k) *q++ = names[k];
    *q = (i + 1 == e) ? '\n' : ',';
}

// final.txt (src/run.sh:16-20): every line of every mr-{r}.txt, sorted bytewise.  Keys are distinct
// across partitions and their bytes are all > ' ', so the line order is the key order; the only keys
// missing are those the per-partition pass dropped (the last group of each partition, worker.rs:
// 169-184).  part2[key] = 1 for those, 0 for the rest; a sort by (part2, key) then puts final.txt in
// "partition" 0.  r is sorted by (partition, full key bytes[, doc]).
__global__ void k_final_part(const SortRec *r, uint64_t n, KeySet ks, const uint8_t *heap, int drop_last,
                             uint32_t *part2) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t e = i + 1;  // first record of the next group (indexer groups span several docs)
    while (e < n && same_key(r[i], r[e], ks, heap)) ++e;
    const bool dropped = drop_last && (e == n || r[e].part != r[i].part);
    part2[r[i].idx] = dropped ? 1u : 0u;
}

__global__ void k_gather_first(const SortRec *r, const uint64_t *H, uint64_t G, SortRec *out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g < G) out[g] = r[H[g]];
}

}  // namespace

void mrg_launch_fix_runs(SortRec *r, uint64_t n, KeySet ks, const uint8_t *heap, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_fix_runs, grid_for(n), dim3(256), 0, s, r, n, ks, heap);
}

void mrg_launch_final_part(const SortRec *r, uint64_t n, KeySet ks, const uint8_t *heap, int drop_last,
                           uint32_t *part2, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_final_part, grid_for(n), dim3(256), 0, s, r, n, ks, heap, drop_last, part2);
}

uint64_t mrg_format(const FormatArgs &f, DevPool &pool, uint8_t **out_buf, uint64_t *out_cap,
                    uint64_t *part_off_host, hipStream_t s) {
    const uint64_t n = f.n;
    const uint32_t R = f.n_reduce;
    SortRec *recs = const_cast<SortRec *>(f.recs);
    uint64_t *part_off = (uint64_t *)pool.get(sizeof(uint64_t) * (R + 1));
    uint64_t *total_d = (uint64_t *)pool.get(sizeof(uint64_t) * 2);
    // (no memset: k_part_off writes every entry 0..R, also for n == 0)
    uint64_t *scantmp = (uint64_t *)pool.get(sizeof(uint64_t) * mrg_scan_tmp_elems(n + 1));
    if (n && f.any_long) hipLaunchKernelGGL(k_fix_runs, grid_for(n), dim3(256), 0, s, recs, n, f.ks, f.heap);

    uint64_t total = 0;
    if (!f.indexer) {
        uint64_t *L = (uint64_t *)pool.get(sizeof(uint64_t) * (n + 1));
        uint64_t *O = (uint64_t *)pool.get(sizeof(uint64_t) * (n + 1));
        if (n) {
            hipLaunchKernelGGL(k_wc_len, grid_for(n), dim3(256), 0, s, recs, n, f.ks, f.drop_last, f.carried, L);
            mrg_scan_u64(L, O, n, scantmp, s);
        }
        hipLaunchKernelGGL(k_total, dim3(1), dim3(1), 0, s, L, O, n, total_d);
        // no round trip for the byte count: the buffer is sized by a bound ("key count\n" with at most
        // 16 short-key bytes or the long key's heap bytes, and 20 digits), the count read with part_off
        const uint64_t bound = n * (16u + 2u + 20u) + f.heap_bytes + 16u;
        if (bound > *out_cap) {
            if (*out_buf) pool.put(*out_buf);
            *out_cap = bound;
            *out_buf = (uint8_t *)pool.get(*out_cap);
        }
        if (n)
            hipLaunchKernelGGL(k_wc_write, grid_for(n), dim3(256), 0, s, recs, n, f.ks, f.heap, L, O, f.carried, *out_buf);
        hipLaunchKernelGGL(k_part_off, grid_for(n + 1), dim3(256), 0, s, recs, O, n, R, (const uint64_t *)nullptr,
                           (const uint64_t *)total_d, part_off);
        hipMemcpyAsync(&total, total_d, sizeof total, hipMemcpyDeviceToHost, s);
        pool.put(L);
        pool.put(O);
    } else {
        uint64_t *head = (uint64_t *)pool.get(sizeof(uint64_t) * (n + 1));
        uint64_t *E = (uint64_t *)pool.get(sizeof(uint64_t) * (n + 1));
        uint64_t *nl = (uint64_t *)pool.get(sizeof(uint64_t) * (n + 1));
        uint64_t *P = (uint64_t *)pool.get(sizeof(uint64_t) * (n + 1));
        uint64_t G = 0, Ptot = 0;
        if (n) {
            hipLaunchKernelGGL(k_idx_heads, grid_for(n), dim3(256), 0, s, recs, n, f.ks, f.heap, f.name_off, head, nl);
            mrg_scan_u64(head, E, n, scantmp, s);
            mrg_scan_u64(nl, P, n, scantmp, s);
            hipLaunchKernelGGL(k_total, dim3(1), dim3(1), 0, s, head, E, n, total_d);
            hipLaunchKernelGGL(k_total, dim3(1), dim3(1), 0, s, nl, P, n, total_d + 1);
            uint64_t tt[2];
            hipMemcpyAsync(tt, total_d, sizeof tt, hipMemcpyDeviceToHost, s);
            hipStreamSynchronize(s);
            G = tt[0];
            Ptot = tt[1];
        }
        uint64_t *H = (uint64_t *)pool.get(sizeof(uint64_t) * (G + 1));
        uint64_t *GL = (uint64_t *)pool.get(sizeof(uint64_t) * (G + 1));
        uint64_t *GO = (uint64_t *)pool.get(sizeof(uint64_t) * (G + 1));
        SortRec *first = (SortRec *)pool.get(sizeof(SortRec) * (G + 1));
        if (G) {
            hipLaunchKernelGGL(k_idx_groups, grid_for(n), dim3(256), 0, s, head, E, n, H);
            hipLaunchKernelGGL(k_idx_glen, grid_for(G), dim3(256), 0, s, recs, n, G, f.ks, H, P, Ptot, f.drop_last, GL);
            mrg_scan_u64(GL, GO, G, scantmp, s);
        }
        hipLaunchKernelGGL(k_total, dim3(1), dim3(1), 0, s, GL, GO, G, total_d);
        hipMemcpyAsync(&total, total_d, sizeof total, hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
        if (total + 16 > *out_cap) {
            if (*out_buf) pool.put(*out_buf);
            *out_cap = total + 16;
            *out_buf = (uint8_t *)pool.get(*out_cap);
        }
        if (n)
            hipLaunchKernelGGL(k_idx_write, grid_for(n), dim3(256), 0, s, recs, n, G, f.ks, f.heap, head, E, H, P, GL,
                               GO, f.names, f.name_off, *out_buf);
        if (G) hipLaunchKernelGGL(k_gather_first, grid_for(G), dim3(256), 0, s, recs, H, G, first);
        hipLaunchKernelGGL(k_part_off, grid_for(G + 1), dim3(256), 0, s, first, GO, G, R, (const uint64_t *)nullptr,
                           (const uint64_t *)total_d, part_off);
        pool.put(head); pool.put(E); pool.put(nl); pool.put(P);
        pool.put(H); pool.put(GL); pool.put(GO); pool.put(first);
    }
    hipMemcpyAsync(part_off_host, part_off, sizeof(uint64_t) * (R + 1), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    pool.put(part_off);
    pool.put(total_d);
    pool.put(scantmp);
    return total;
}
