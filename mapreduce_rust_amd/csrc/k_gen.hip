// k_gen.hip -- synthetic benchmark inputs, generated in HBM (NOT on the data path).
//
// C3/C4 (BASELINE.json configs[2], [3]): Zipf(s) text over a vocabulary of V distinct lowercase
// words.  Word r = splitmix64 stream of (seed, r): length 2..12, letters a-z, duplicates re-drawn
// (host, deterministic).  Token j of file f: rank drawn i.i.d. Zipf(s) by a Vose alias table from
// splitmix64(seed, f, j); 5% of tokens get a trailing mark from ".,;:!?" and 2% an inner apostrophe
// (exercises wc.rs's delete-and-join); ' ' between tokens, '\n' after every 12th.  Tokens are laid
// out by an exclusive scan of their lengths; the file is filled up to n_bytes with whole tokens and
// padded with '\n'.
// Style 1 ("zipf_u", Gutenberg-like Unicode; the reference corpus src/data/gut-*.txt has one non-ASCII
// codepoint per ~190 bytes in its larger files, mostly U+2019/201C/201D/2014 and Latin-1 letters): the
// same tokens, with the inner apostrophe written as U+2019, 1.5 % of tokens opened by U+201C and 1.5 %
// closed by U+201D (deleted: not \w), 0.3 % followed by U+2014 instead of the separator (deleted, so
// the two words join into one key) and 0.3 % with one letter replaced by U+00E9 (\w, a 2-byte key byte
// pair).  About one non-ASCII codepoint per 150 bytes: nearly every 1 KiB tile holds one.
// C5: near-unique keys: token i = 12 chars of [a-z0-9] from splitmix64(seed + i), 1% copies of an
// earlier token.
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <unordered_set>
#include <vector>

#include "mrg_device.h"
#include "mrg_internal.h"

namespace {

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct ZipfDev {
    const uint8_t *vocab;      // concatenated words
    const uint32_t *voff;      // [V + 1]
    const uint32_t *prob;      // alias threshold (2^32 scale)
    const uint32_t *alias;
    uint32_t V;
    uint64_t seed, file;
    uint32_t style;  // 0 ASCII, 1 Gutenberg-like Unicode
};

struct Tok {
    uint32_t w, len, punct, apos;  // punct: 0 or char; apos: 0 or position
    uint32_t oq, cq, dash, acc;    // style 1: U+201C before, U+201D after, U+2014 as separator, U+00E9 at acc - 1
};

__device__ inline Tok zipf_token(const ZipfDev &z, uint64_t j) {
    const uint64_t x = splitmix64(z.seed ^ splitmix64(z.file * 0xD1B54A32D192ED03ull + j));
    const uint32_t i = (uint32_t)(((x >> 32) * (uint64_t)z.V) >> 32);
    const uint32_t u = (uint32_t)x;
    Tok t;
    t.w = u < z.prob[i] ? i : z.alias[i];
    const uint32_t wl = z.voff[t.w + 1] - z.voff[t.w];
    const uint64_t y = splitmix64(x);
    const uint32_t pr = (uint32_t)(y % 10000u);
    t.punct = pr < 500u ? (uint32_t)".,;:!?"[(y >> 20) % 6u] : 0u;
    const uint32_t ar = (uint32_t)((y >> 40) % 10000u);
    t.apos = (ar < 200u && wl >= 2u) ? 1u + (uint32_t)((y >> 8) % (wl - 1u)) : 0u;
    t.len = wl + (t.punct ? 1u : 0u) + (t.apos ? 1u : 0u) + 1u;  // + separator
    t.oq = t.cq = t.dash = t.acc = 0;
    if (z.style == 1) {
        const uint64_t u2 = splitmix64(y);
        t.oq = (uint32_t)(u2 % 10000u) < 150u;
        t.cq = (uint32_t)((u2 >> 14) % 10000u) < 150u;
        t.dash = (uint32_t)((u2 >> 28) % 10000u) < 30u;
        t.acc = (uint32_t)((u2 >> 42) % 10000u) < 30u ? 1u + (uint32_t)((u2 >> 56) % wl) : 0u;
        // U+2019 is 3 bytes (the ASCII apostrophe was 1), the quotes 3 each, U+2014 replaces the 1-byte
        // separator, U+00E9 replaces one letter
        t.len += (t.apos ? 2u : 0u) + 3u * (t.oq + t.cq) + (t.dash ? 2u : 0u) + (t.acc ? 1u : 0u);
    }
    return t;
}

__global__ void k_zipf_len(ZipfDev z, uint64_t J, uint64_t *len) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < J) len[j] = zipf_token(z, j).len;
}

__global__ void k_zipf_write(ZipfDev z, uint64_t J, const uint64_t *off, uint8_t *dst, uint64_t n) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= J) return;
    const Tok t = zipf_token(z, j);
    const uint64_t o = off[j];
    if (o + t.len > n) return;
    uint8_t *p = dst + o;
    const uint32_t a = z.voff[t.w], wl = z.voff[t.w + 1] - a;
    auto put3 = [&](uint32_t b2) { p[0] = 0xE2; p[1] = 0x80; p[2] = (uint8_t)b2; p += 3; };
    if (t.oq) put3(0x9C);  // U+201C
    for (uint32_t k = 0; k < wl; ++k) {
        if (t.apos && k == t.apos) {
            if (z.style == 1) put3(0x99);  // U+2019
            else *p++ = '\'';
        }
        if (t.acc && k == t.acc - 1) { p[0] = 0xC3; p[1] = 0xA9; p += 2; }  // U+00E9
        else *p++ = z.vocab[a + k];
    }
    if (t.punct) *p++ = (uint8_t)t.punct;
    if (t.cq) put3(0x9D);  // U+201D
    if (t.dash) put3(0x94);  // U+2014 instead of the separator
    else *p = (j % 12u == 11u) ? '\n' : ' ';
}

__global__ void k_unique_write(uint8_t *dst, uint64_t n, uint64_t seed, uint64_t first, uint64_t J) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= J) return;
    uint64_t g = first + j;
    const uint64_t y = splitmix64(seed * 0x2545F4914F6CDD1Dull ^ g);
    if (g > 0 && (y % 100u) == 0u) g = g - 1u - (y >> 8) % (g < 1000000u ? g : 1000000u);  // 1% repeats
    uint64_t x = splitmix64(seed + g);
    uint64_t x2 = splitmix64(x);
    uint8_t *p = dst + j * 13u;
    for (int k = 0; k < 12; ++k) {
        const uint64_t src = k < 6 ? x : x2;
        const uint32_t c = (uint32_t)((src >> (10 * (k % 6))) & 1023u) % 36u;
        p[k] = (uint8_t)(c < 26u ? 'a' + c : '0' + (c - 26u));
    }
    p[12] = (j % 12u == 11u) ? '\n' : ' ';
}

// Host vocabulary + alias table cache (per process; rebuilt when (seed, V, s) changes)
struct ZipfHost {
    uint64_t seed = 0;
    uint32_t V = 0;
    double s = 0;
    uint8_t *d_vocab = nullptr;
    uint32_t *d_voff = nullptr, *d_prob = nullptr, *d_alias = nullptr;
};
ZipfHost g_zipf;

int build_zipf(uint64_t seed, uint32_t V, double s) {
    if (g_zipf.d_vocab && g_zipf.seed == seed && g_zipf.V == V && g_zipf.s == s) return 0;
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> off(1, 0);
    std::unordered_set<std::string> seen;
    seen.reserve(V * 2);
    uint64_t ctr = 0;
    while (off.size() <= V) {
        const uint64_t x = splitmix64(seed ^ splitmix64(0xC0FFEEull + ctr++));
        const uint32_t len = 2u + (uint32_t)(x % 11u);
        std::string w(len, 'a');
        uint64_t y = splitmix64(x);
        for (uint32_t k = 0; k < len; ++k) w[k] = (char)('a' + (y >> (5 * k)) % 26u);
        if (!seen.insert(w).second) continue;
        bytes.insert(bytes.end(), w.begin(), w.end());
        off.push_back((uint32_t)bytes.size());
    }
    // Vose alias table for p(r) ~ (r+1)^-s
    std::vector<double> p(V);
    double tot = 0;
    for (uint32_t r = 0; r < V; ++r) tot += (p[r] = std::pow((double)r + 1.0, -s));
    std::vector<double> q(V);
    std::vector<uint32_t> small, large, alias(V, 0), prob(V, 0);
    for (uint32_t r = 0; r < V; ++r) {
        q[r] = p[r] / tot * V;
        (q[r] < 1.0 ? small : large).push_back(r);
    }
    while (!small.empty() && !large.empty()) {
        const uint32_t a = small.back(); small.pop_back();
        const uint32_t b = large.back(); large.pop_back();
        prob[a] = (uint32_t)std::min(4294967295.0, q[a] * 4294967296.0);
        alias[a] = b;
        q[b] = (q[b] + q[a]) - 1.0;
        (q[b] < 1.0 ? small : large).push_back(b);
    }
    for (uint32_t r : large) { prob[r] = 0xFFFFFFFFu; alias[r] = r; }
    for (uint32_t r : small) { prob[r] = 0xFFFFFFFFu; alias[r] = r; }
    if (g_zipf.d_vocab) {
        (void)hipFree(g_zipf.d_vocab); (void)hipFree(g_zipf.d_voff);
        (void)hipFree(g_zipf.d_prob); (void)hipFree(g_zipf.d_alias);
    }
    if (hipMalloc(&g_zipf.d_vocab, bytes.size() + 16) != hipSuccess) return -1;
    if (hipMalloc(&g_zipf.d_voff, off.size() * 4) != hipSuccess) return -1;
    if (hipMalloc(&g_zipf.d_prob, V * 4ull) != hipSuccess) return -1;
    if (hipMalloc(&g_zipf.d_alias, V * 4ull) != hipSuccess) return -1;
    hipMemcpy(g_zipf.d_vocab, bytes.data(), bytes.size(), hipMemcpyHostToDevice);
    hipMemcpy(g_zipf.d_voff, off.data(), off.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(g_zipf.d_prob, prob.data(), V * 4ull, hipMemcpyHostToDevice);
    hipMemcpy(g_zipf.d_alias, alias.data(), V * 4ull, hipMemcpyHostToDevice);
    g_zipf.seed = seed; g_zipf.V = V; g_zipf.s = s;
    return 0;
}

}  // namespace

int mrg_gen_zipf_impl(uint8_t *dst, uint64_t n, uint64_t seed, uint64_t file_index, uint32_t vocab, double s,
                      uint32_t style, hipStream_t st) {
    if (vocab < 1 || s <= 0 || style > 1) return -1;
    if (build_zipf(seed, vocab, s)) return -1;
    ZipfDev z{g_zipf.d_vocab, g_zipf.d_voff, g_zipf.d_prob, g_zipf.d_alias, vocab, seed, file_index, style};
    const uint64_t J = n / 3 + 2;  // every token is >= 3 bytes: J tokens always overfill n bytes
    uint64_t *len = nullptr, *off = nullptr, *tmp = nullptr;
    if (hipMalloc(&len, J * 8) != hipSuccess) return -1;
    if (hipMalloc(&off, J * 8) != hipSuccess) return -1;
    if (hipMalloc(&tmp, mrg_scan_tmp_elems(J) * 8) != hipSuccess) return -1;
    const unsigned g = (unsigned)((J + 255) / 256);
    hipMemsetAsync(dst, '\n', n, st);
    hipLaunchKernelGGL(k_zipf_len, dim3(g), dim3(256), 0, st, z, J, len);
    mrg_scan_u64(len, off, J, tmp, st);
    hipLaunchKernelGGL(k_zipf_write, dim3(g), dim3(256), 0, st, z, J, off, dst, n);
    hipStreamSynchronize(st);
    (void)hipFree(len); (void)hipFree(off); (void)hipFree(tmp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int mrg_gen_unique_impl(uint8_t *dst, uint64_t n, uint64_t seed, uint64_t file_index, hipStream_t st) {
    const uint64_t J = n / 13u;
    hipMemsetAsync(dst, '\n', n, st);
    if (J) {
        const uint64_t first = file_index * J;  // files of equal size -> disjoint index ranges
        hipLaunchKernelGGL(k_unique_write, dim3((unsigned)((J + 255) / 256)), dim3(256), 0, st, dst, n, seed, first, J);
    }
    hipStreamSynchronize(st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
