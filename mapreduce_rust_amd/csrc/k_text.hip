// k_text.hip -- the reference's text intermediates, byte for byte, gfx950.
//
// Writer: Worker::write_key_value_to_file (src/mr/worker.rs:117-140) appends "{key} {value}\n" for
// every KeyValue that wc::map (src/app/wc.rs:6-13) produced, in input order, to mr-{m}-{r}.txt with
// r = SipHash-1-3(key ++ 0xFF) % nReduce (worker.rs:111-115, 129).  Here: every thread walks the
// codepoints of one 64-byte segment of the input (exact UTF-8 decode + the \w / White_Space class
// table), emits the tokens that START in its segment as (packed key, raw range, key length,
// partition) records -- a count pass, a scan, an emit pass -- then a stable radix sort by partition
// keeps input order inside each partition and every record is written as "key 1\n" at its offset.
//
// Reader: Worker::read_file_to_mem_reduce (worker.rs:79-109): read_to_string (UTF-8 validated),
// split("\n"), drop empty lines, split(" ") must give exactly two fields (assert!), key = field 0.
// Here: UTF-8 validation by byte, then one thread per 64-byte segment parses the lines that start in
// it into exchange records (count 1, key bytes verbatim in the text buffer); the reduce loop then
// counts values per key (wc::reduce = values.len(), wc.rs:15-17).
#include "mrg_device.h"
#include "mrg_internal.h"

namespace {

constexpr uint64_t SEGB = 64;  // bytes per thread

inline dim3 grid_for(uint64_t n, int b = 256) { return dim3((unsigned)((n + b - 1) / b)); }

__device__ __forceinline__ void report(unsigned long long *err, uint64_t pos) {
    atomicMin(err, (unsigned long long)pos);
}

// <str as Hash>::hash + DefaultHasher::finish over bytes pushed one at a time (key ++ 0xFF)
struct SipStream {
    MrgSip s;
    uint64_t buf = 0;
    uint32_t nb = 0;
    uint64_t tot = 0;
    __device__ __forceinline__ void push(uint32_t b) {
        buf |= (uint64_t)(b & 0xFFu) << (8u * nb);
        ++tot;
        if (++nb == 8u) {
            s.word(buf);
            buf = 0;
            nb = 0;
        }
    }
    __device__ __forceinline__ uint64_t fin() {
        const uint64_t total = tot + 1u;  // the 0xFF terminator counts
        buf |= 0xFFull << (8u * nb);
        if (++nb == 8u) {
            s.word(buf);
            return s.finish(0ull, total);
        }
        return s.finish(buf, total);
    }
};

// ---------------------------------------------------------------- writer (map side)
struct Cursor {  // first codepoint boundary >= s0 and whether the codepoint before it is White_Space
    uint64_t p;
    bool prevS;
    bool bad;
};

template <class RD>
__device__ Cursor seg_start(const RD &rd, uint64_t s0, uint64_t n, unsigned long long *err) {
    Cursor c{s0, true, false};
    if (s0 == 0) return c;
    uint32_t j = 0;  // continuation bytes here belong to a codepoint that starts before s0
    while (j < 3 && s0 + j < n && mrg_is_cont(rd(s0 + j))) ++j;
    c.p = s0 + j;
    uint32_t k = 1;  // lead of the codepoint ending at p - 1
    while (k <= 3 && c.p >= k + 1 && mrg_is_cont(rd(c.p - k))) ++k;
    if (c.p < k || mrg_is_cont(rd(c.p - k))) {  // orphan continuation bytes
        report(err, s0);
        c.bad = true;
        return c;
    }
    const uint64_t q = c.p - k;
    uint32_t cp, raw;
    const int l = mrg_utf8_decode(rd, q, n, &cp, &raw);
    if (l == 0 || q + (uint64_t)l != c.p) {
        report(err, s0);
        c.bad = true;
        return c;
    }
    c.prevS = mrg_uclass(cp) == MRG_CLS_S;
    return c;
}

// Count (out == null) or emit the tokens starting in each 64-byte segment.
__global__ void k_text_tok(const uint8_t *in, uint64_t n, uint32_t n_reduce, const uint64_t *base, uint64_t *cnt,
                           TextTok *out, unsigned long long *err) {
    const uint64_t seg = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t s0 = seg * SEGB;
    if (s0 >= n) return;
    const uint64_t s1 = min(s0 + SEGB, n);
    auto rd = [&](uint64_t x) -> uint32_t { return in[x]; };
    Cursor c = seg_start(rd, s0, n, err);
    uint64_t k = 0, o = out ? base[seg] : 0;
    uint64_t p = c.p;
    bool prevS = c.prevS;
    while (!c.bad && p < s1) {
        uint32_t cp, raw;
        const int l = mrg_utf8_decode(rd, p, n, &cp, &raw);
        if (!l) {
            report(err, p);
            break;
        }
        const uint32_t cl = mrg_uclass(cp);
        if (cl == MRG_CLS_S) {
            prevS = true;
            p += (uint64_t)l;
            continue;
        }
        if (!prevS) {
            p += (uint64_t)l;
            continue;
        }
        // a token starts at p: keep its \w bytes up to the next White_Space (wc.rs:7-10)
        const uint64_t a = p;
        uint64_t k0 = 0, k1 = 0;
        uint32_t L = 0;
        SipStream h;
        bool ok = true;
        while (p < n) {
            uint32_t cp2, raw2;
            const int l2 = mrg_utf8_decode(rd, p, n, &cp2, &raw2);
            if (!l2) {
                report(err, p);
                ok = false;
                break;
            }
            const uint32_t c2 = mrg_uclass(cp2);
            if (c2 == MRG_CLS_S) break;
            if (c2 == MRG_CLS_W)
                for (int b = 0; b < l2; ++b) {
                    const uint32_t by = (raw2 >> (8 * b)) & 0xFFu;
                    mrg_key_append(k0, k1, L, by);
                    h.push(by);
                    ++L;
                }
            p += (uint64_t)l2;
        }
        if (!ok) break;
        prevS = false;
        if (L == 0) continue;  // only deleted codepoints: split_whitespace yields nothing
        if (out) {
            TextTok t;
            t.k0 = k0;
            t.k1 = k1;
            t.start = a;
            t.rawlen = (uint32_t)(p - a);
            t.klen = L;
            t.part = (uint32_t)(h.fin() % (uint64_t)n_reduce);
            t.pad = 0;
            out[o + k] = t;
        }
        ++k;
    }
    if (!out) cnt[seg] = k;
}

__global__ void k_text_keys(const TextTok *t, uint64_t n, uint64_t *part, uint32_t *idx) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    part[i] = t[i].part;
    idx[i] = (uint32_t)i;
}

__global__ void k_text_len(const TextTok *t, const uint32_t *idx, uint64_t n, uint64_t *L) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) L[i] = (uint64_t)t[idx[i]].klen + 3u;  // "key 1\n"
}

// part_off[r] = first byte of partition r (parts sorted ascending); part_off[R] = total
__global__ void k_text_part_off(const uint64_t *part, const uint64_t *O, uint64_t n, uint32_t R, uint64_t total,
                                uint64_t *part_off) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const int64_t prev = i == 0 ? -1 : (int64_t)part[i - 1];
    const int64_t cur = i == n ? (int64_t)R : (int64_t)part[i];
    for (int64_t r = prev + 1; r <= cur; ++r) part_off[r] = i == n ? total : O[i];
}

__global__ void k_text_write(const uint8_t *in, const TextTok *t, const uint32_t *idx, uint64_t n, const uint64_t *O,
                             uint8_t *outb) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const TextTok x = t[idx[i]];
    uint8_t *o = outb + O[i];
    if (x.klen <= 16u) {
        for (uint32_t b = 0; b < x.klen; ++b) o[b] = (uint8_t)mrg_key_byte(x.k0, x.k1, b);
        o += x.klen;
    } else {  // re-walk the raw token, keeping \w codepoints
        auto rd = [&](uint64_t q) -> uint32_t { return in[q]; };
        const uint64_t e = x.start + x.rawlen;
        for (uint64_t p = x.start; p < e;) {
            uint32_t cp, raw;
            int l = mrg_utf8_decode(rd, p, e, &cp, &raw);
            if (!l) l = 1;  // validated by k_text_tok
            if (mrg_uclass(cp) == MRG_CLS_W)
                for (int b = 0; b < l; ++b) *o++ = (uint8_t)(raw >> (8 * b));
            p += (uint64_t)l;
        }
    }
    o[0] = ' ';
    o[1] = '1';
    o[2] = '\n';
}

// ---------------------------------------------------------------- reader (reduce side)
// str::from_utf8 acceptance by byte: a lead byte's sequence must decode; a continuation byte must
// be covered by the sequence of the nearest lead at most 3 bytes before it.
__global__ void k_utf8_check(const uint8_t *in, uint64_t n, unsigned long long *err) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t b = in[i];
    if (b < 0x80u) return;
    auto rd = [&](uint64_t x) -> uint32_t { return in[x]; };
    if (!mrg_is_cont(b)) {
        uint32_t cp, raw;
        if (!mrg_utf8_decode(rd, i, n, &cp, &raw)) report(err, i);
        return;
    }
    uint32_t k = 1;
    while (k <= 3 && i >= k && mrg_is_cont(in[i - k])) ++k;
    if (k > 3 || i < k) {
        report(err, i);
        return;
    }
    const int L = mrg_utf8_len(in[i - k]);
    if ((uint32_t)L <= k) report(err, i);
}

// Lines starting in each 64-byte segment of file f ([fo[f], fe[f]) of the buffer; files start on
// 64-byte boundaries, so a segment lies in one file): count pass
// (out == null) or emit one exchange record per non-empty line with a non-empty key.  A line must
// have exactly one ' ' (worker.rs:100 assert!); a key with a NUL byte has no packed form (the
// reference's map never writes one): both are reported in err[1].  Lines with an empty key are
// counted in nempty (the reduce loop folds them into the next group, see mrgpu.cpp).
__global__ void k_text_lines(const uint8_t *in, const uint64_t *fo, const uint64_t *fe, uint32_t nf, uint64_t nseg,
                             const uint64_t *base, uint64_t *cnt, LRec *out, unsigned long long *err,
                             unsigned long long *nempty) {
    const uint64_t seg = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (seg >= nseg) return;
    const uint64_t s0 = seg * SEGB;
    uint32_t lo = 0, hi = nf;  // file of this segment: the last f with fo[f] <= s0
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (fo[mid] <= s0) lo = mid;
        else hi = mid;
    }
    const uint64_t fbeg = fo[lo], fend = fe[lo];
    const uint64_t s1 = min(s0 + SEGB, fend);
    uint64_t k = 0, o = out ? base[seg] : 0;
    for (uint64_t a = s0; a < s1; ++a) {
        if (a != fbeg && in[a - 1] != '\n') continue;  // not a line start
        uint64_t e = a, sp = ~0ull;
        uint32_t nsp = 0;
        while (e < fend && in[e] != '\n') {
            if (in[e] == ' ') {
                if (!nsp) sp = e;
                ++nsp;
            }
            ++e;
        }
        if (e == a) continue;  // empty line (filter(|x| !x.is_empty()))
        if (nsp != 1) {
            report(err + 1, a);
            continue;
        }
        const uint32_t klen = (uint32_t)(sp - a);
        if (klen == 0) {
            if (out) atomicAdd(nempty, 1ull);
            continue;
        }
        uint64_t k0 = 0, k1 = 0;
        bool nul = false;
        for (uint32_t b = 0; b < klen; ++b) {
            const uint32_t by = in[a + b];
            nul |= by == 0u;
            if (b < 16u) mrg_key_append(k0, k1, b, by);
        }
        if (nul) {
            report(err + 1, a);
            continue;
        }
        if (out) {
            LRec x;
            x.k0 = k0;
            x.k1 = k1;
            x.cnt = 1;
            x.doc = MRG_EMPTY_DOC;
            x.len = klen;
            x.heap = klen > 16u ? a - fbeg : MRG_NO_HEAP;  // key bytes in this file's segment
            out[o + k] = x;
        }
        ++k;
    }
    if (!out) cnt[seg] = k;
}

__global__ void k_add_first(const SortRec *r, KeySet ks, uint64_t v) { ks.cnt[r[0].idx] += v; }

}  // namespace

void mrg_launch_text_tok(const uint8_t *in, uint64_t n, uint32_t n_reduce, const uint64_t *base, uint64_t *cnt,
                         TextTok *out, unsigned long long *err, hipStream_t s) {
    const uint64_t nseg = (n + SEGB - 1) / SEGB;
    if (nseg) hipLaunchKernelGGL(k_text_tok, grid_for(nseg), dim3(256), 0, s, in, n, n_reduce, base, cnt, out, err);
}
uint64_t mrg_text_segments(uint64_t n) { return (n + SEGB - 1) / SEGB; }
void mrg_launch_text_keys(const TextTok *t, uint64_t n, uint64_t *part, uint32_t *idx, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_text_keys, grid_for(n), dim3(256), 0, s, t, n, part, idx);
}
void mrg_launch_text_len(const TextTok *t, const uint32_t *idx, uint64_t n, uint64_t *L, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_text_len, grid_for(n), dim3(256), 0, s, t, idx, n, L);
}
void mrg_launch_text_part_off(const uint64_t *part, const uint64_t *O, uint64_t n, uint32_t R, uint64_t total,
                              uint64_t *part_off, hipStream_t s) {
    hipLaunchKernelGGL(k_text_part_off, grid_for(n + 1), dim3(256), 0, s, part, O, n, R, total, part_off);
}
void mrg_launch_text_write(const uint8_t *in, const TextTok *t, const uint32_t *idx, uint64_t n, const uint64_t *O,
                           uint8_t *out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_text_write, grid_for(n), dim3(256), 0, s, in, t, idx, n, O, out);
}
void mrg_launch_utf8_check(const uint8_t *in, uint64_t n, unsigned long long *err, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_utf8_check, grid_for(n), dim3(256), 0, s, in, n, err);
}
void mrg_launch_text_lines(const uint8_t *in, const uint64_t *fo, const uint64_t *fe, uint32_t nf, uint64_t nseg,
                           const uint64_t *base, uint64_t *cnt, LRec *out, unsigned long long *err,
                           unsigned long long *nempty, hipStream_t s) {
    if (nseg)
        hipLaunchKernelGGL(k_text_lines, grid_for(nseg), dim3(256), 0, s, in, fo, fe, nf, nseg, base, cnt, out, err,
                           nempty);
}
void mrg_launch_add_first(const SortRec *r, KeySet ks, uint64_t v, hipStream_t s) {
    hipLaunchKernelGGL(k_add_first, dim3(1), dim3(1), 0, s, r, ks, v);
}
