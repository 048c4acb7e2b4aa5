/*
 * oracle.c -- CPU restatement of the Freebirdgo/MapReduce_Rust worker data path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this library, and only as the checker / the reported CPU baseline.  The product path
 * (mapreduce_rust_amd/, libmrgpu.so) never links or calls it.
 *
 * Parity pin: the reference is Rust and cannot be built here (no toolchain), so this
 * restatement is pinned by (1) the C1 digests of SURVEY.md §8(c), reproduced by the Python twin
 * tests/golden/twin.py and committed in tests/golden/golden.json, (2) the SipHash paper vectors,
 * (3) tokenizer known-answer cases.  tests/test_oracle.py checks all three.
 *
 * What it restates (file:line in /root/reference):
 *   wc::map             src/app/wc.rs:6-13      [^\w\s] deleted, split_whitespace, emit (tok,"1")
 *   wc::reduce          src/app/wc.rs:15-17     count of values
 *   read_to_string      src/mr/worker.rs:65-77  UTF-8 validated (invalid -> panic; here: error code)
 *   cal_hash_for_key    src/mr/worker.rs:111-115  SipHash-1-3 k=(0,0) over key bytes ++ 0xFF
 *   write_key_value_to_file  worker.rs:117-140  one "k 1\n" write per token to mr-{m}-{h%R}.txt
 *   read_file_to_mem_reduce  worker.rs:79-109   parse mr-{m}-{r}.txt for m in 0..map_n
 *   Worker::reduce      worker.rs:157-193       stable byte-order sort, group, last group dropped
 *
 * Two modes produce byte-identical outputs:
 *   ORACLE_FAITHFUL : the reference's structure (per-token write(2) + log line, files, read-back,
 *                     stable sort of every record, adjacent grouping) -- the "reference CPU path"
 *   ORACLE_FAST     : in-memory hash count + sort of distinct keys (a checker at larger sizes)
 * and two multi-threaded forms of them:
 *   oracle_wc_workers : FAITHFUL with W worker threads that pull map task ids, then reduce task ids,
 *                       like W `mrworker` processes under the coordinator (mrworker.rs:43-149,
 *                       coordinator.rs:137-215) -- the CPU baseline at W = host cores
 *   oracle_wc_mt      : FAST over whitespace-aligned chunks on T threads (the full-size checker)
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include "uclass_ranges.inc"

#define ORACLE_OK 0
#define ORACLE_EUTF8 (-2)
#define ORACLE_EIO (-3)
#define ORACLE_EARG (-4)

enum { ORACLE_FAITHFUL = 0, ORACLE_FAST = 1 };

/* ------------------------------------------------------------------ classes (wc.rs:7-10) */

/* 0 = X (deleted by [^\w\s]), 1 = W (\w), 2 = S (White_Space) */
int oracle_class(uint32_t cp) {
    int lo = 0, hi = ORACLE_NRUNS - 1;
    while (lo <= hi) {
        int mid = (lo + hi) / 2;
        if (cp < ORACLE_RUNS[mid][0]) hi = mid - 1;
        else if (cp > ORACLE_RUNS[mid][1]) lo = mid + 1;
        else return (int)ORACLE_RUNS[mid][2];
    }
    return 0;
}

/* ------------------------------------------------------------------ UTF-8 (worker.rs:75) */

/* Decode one scalar at s[i..n).  Returns its byte length (1..4) and sets *cp, or 0 if invalid
 * (the same acceptance as Rust's str::from_utf8: no overlongs, no surrogates, <= U+10FFFF). */
static int utf8_next(const uint8_t *s, size_t n, size_t i, uint32_t *cp) {
    uint8_t b0 = s[i];
    if (b0 < 0x80) { *cp = b0; return 1; }
    if (b0 < 0xC2) return 0;
    if (b0 < 0xE0) {
        if (i + 1 >= n || (s[i + 1] & 0xC0) != 0x80) return 0;
        *cp = ((uint32_t)(b0 & 0x1F) << 6) | (s[i + 1] & 0x3F);
        return 2;
    }
    if (b0 < 0xF0) {
        if (i + 2 >= n) return 0;
        uint8_t b1 = s[i + 1], b2 = s[i + 2];
        if ((b1 & 0xC0) != 0x80 || (b2 & 0xC0) != 0x80) return 0;
        if (b0 == 0xE0 && b1 < 0xA0) return 0;          /* overlong */
        if (b0 == 0xED && b1 >= 0xA0) return 0;         /* surrogate */
        *cp = ((uint32_t)(b0 & 0x0F) << 12) | ((uint32_t)(b1 & 0x3F) << 6) | (b2 & 0x3F);
        return 3;
    }
    if (b0 < 0xF5) {
        if (i + 3 >= n) return 0;
        uint8_t b1 = s[i + 1], b2 = s[i + 2], b3 = s[i + 3];
        if ((b1 & 0xC0) != 0x80 || (b2 & 0xC0) != 0x80 || (b3 & 0xC0) != 0x80) return 0;
        if (b0 == 0xF0 && b1 < 0x90) return 0;          /* overlong */
        if (b0 == 0xF4 && b1 >= 0x90) return 0;         /* > U+10FFFF */
        *cp = ((uint32_t)(b0 & 0x07) << 18) | ((uint32_t)(b1 & 0x3F) << 12) |
              ((uint32_t)(b2 & 0x3F) << 6) | (b3 & 0x3F);
        return 4;
    }
    return 0;
}

/* ------------------------------------------------------------------ SipHash-1-3 (worker.rs:111-115) */

#define ROTL(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
#define SIPROUND                                                               \
    do {                                                                       \
        v0 += v1; v1 = ROTL(v1, 13); v1 ^= v0; v0 = ROTL(v0, 32);              \
        v2 += v3; v3 = ROTL(v3, 16); v3 ^= v2;                                 \
        v0 += v3; v3 = ROTL(v3, 21); v3 ^= v0;                                 \
        v2 += v1; v1 = ROTL(v1, 17); v1 ^= v2; v2 = ROTL(v2, 32);              \
    } while (0)

/* SipHash-c-d over an arbitrary byte message with a 128-bit key. */
uint64_t oracle_siphash(const uint8_t *m, size_t n, int c, int d, uint64_t k0, uint64_t k1) {
    uint64_t v0 = k0 ^ 0x736f6d6570736575ULL, v1 = k1 ^ 0x646f72616e646f6dULL;
    uint64_t v2 = k0 ^ 0x6c7967656e657261ULL, v3 = k1 ^ 0x7465646279746573ULL;
    size_t full = n & ~(size_t)7;
    for (size_t i = 0; i < full; i += 8) {
        uint64_t w = 0;
        for (int j = 7; j >= 0; --j) w = (w << 8) | m[i + j];
        v3 ^= w;
        for (int r = 0; r < c; ++r) SIPROUND;
        v0 ^= w;
    }
    uint64_t b = (uint64_t)(n & 0xff) << 56;
    for (size_t j = 0; j < n - full; ++j) b |= (uint64_t)m[full + j] << (8 * j);
    v3 ^= b;
    for (int r = 0; r < c; ++r) SIPROUND;
    v0 ^= b;
    v2 ^= 0xff;
    for (int r = 0; r < d; ++r) SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

/* DefaultHasher::new(); key.hash(&mut s); s.finish()  ==  SipHash-1-3(k=0,0) over key ++ 0xFF */
uint64_t oracle_key_hash(const uint8_t *key, size_t len) {
    uint8_t stackbuf[256];
    uint8_t *buf = len + 1 <= sizeof stackbuf ? stackbuf : (uint8_t *)malloc(len + 1);
    memcpy(buf, key, len);
    buf[len] = 0xff;
    uint64_t h = oracle_siphash(buf, len + 1, 1, 3, 0, 0);
    if (buf != stackbuf) free(buf);
    return h;
}

/* ------------------------------------------------------------------ growable buffers */

typedef struct { uint8_t *p; size_t n, cap; } bytes_t;

static void by_reserve(bytes_t *b, size_t extra) {
    if (b->n + extra <= b->cap) return;
    size_t c = b->cap ? b->cap : 4096;
    while (c < b->n + extra) c *= 2;
    b->p = (uint8_t *)realloc(b->p, c);
    b->cap = c;
}
static void by_put(bytes_t *b, const void *src, size_t len) {
    by_reserve(b, len);
    memcpy(b->p + b->n, src, len);
    b->n += len;
}
static void by_putc(bytes_t *b, uint8_t c) { by_reserve(b, 1); b->p[b->n++] = c; }
static void by_putu64(bytes_t *b, uint64_t v) {
    char tmp[24];
    int k = 0;
    do { tmp[k++] = (char)('0' + v % 10); v /= 10; } while (v);
    by_reserve(b, (size_t)k);
    while (k) b->p[b->n++] = (uint8_t)tmp[--k];
}

/* ------------------------------------------------------------------ tokenizer (wc.rs:6-13) */

/* Calls cb(ud, key, len) for every token in input order.  Returns ORACLE_OK or ORACLE_EUTF8.
 * Restatement: delete X codepoints, split on S; a run of W/X with no W yields nothing. */
typedef void (*tok_cb)(void *ud, const uint8_t *key, size_t len);

static int8_t g_ascii_cls[128];
__attribute__((constructor)) static void init_ascii_cls(void) {
    for (uint32_t c = 0; c < 128; ++c) g_ascii_cls[c] = (int8_t)oracle_class(c);
}

static int tokenize(const uint8_t *s, size_t n, tok_cb cb, void *ud, bytes_t *scratch) {
    scratch->n = 0;
    size_t i = 0;
    while (i < n) {
        if (s[i] < 0x80) {  /* ASCII: the class table above (same classes, no decode / search) */
            int c = g_ascii_cls[s[i]];
            if (c == 2) {
                if (scratch->n) { cb(ud, scratch->p, scratch->n); scratch->n = 0; }
            } else if (c == 1) {
                by_putc(scratch, s[i]);
            }
            ++i;
            continue;
        }
        uint32_t cp;
        int l = utf8_next(s, n, i, &cp);
        if (!l) return ORACLE_EUTF8;
        int c = oracle_class(cp);
        if (c == 2) {
            if (scratch->n) { cb(ud, scratch->p, scratch->n); scratch->n = 0; }
        } else if (c == 1) {
            by_put(scratch, s + i, (size_t)l);
        }
        i += (size_t)l;
    }
    if (scratch->n) { cb(ud, scratch->p, scratch->n); scratch->n = 0; }
    return ORACLE_OK;
}

static void cb_stream(void *ud, const uint8_t *k, size_t len) {
    bytes_t *out = (bytes_t *)ud;
    by_put(out, k, len);
    by_putc(out, '\n');
}

/* Token stream "tok\n" per token (tests / fixtures). */
int oracle_tokens(const uint8_t *s, size_t n, uint8_t **out, size_t *out_len) {
    bytes_t o = {0}, scratch = {0};
    int rc = tokenize(s, n, cb_stream, &o, &scratch);
    free(scratch.p);
    if (rc) { free(o.p); return rc; }
    *out = o.p ? o.p : (uint8_t *)malloc(1);
    *out_len = o.n;
    return ORACLE_OK;
}

int oracle_validate_utf8(const uint8_t *s, size_t n, size_t *bad_at) {
    size_t i = 0;
    while (i < n) {
        uint32_t cp;
        int l = utf8_next(s, n, i, &cp);
        if (!l) { if (bad_at) *bad_at = i; return ORACLE_EUTF8; }
        i += (size_t)l;
    }
    return ORACLE_OK;
}

/* ------------------------------------------------------------------ hash map: key bytes -> u64 */

typedef struct { uint64_t h; uint64_t off; uint32_t len; uint64_t val; uint64_t aux; } slot_t;
typedef struct { slot_t *s; size_t cap, n; bytes_t keys; } map_t;

static uint64_t fnv1a(const uint8_t *k, size_t len) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (size_t i = 0; i < len; ++i) { h ^= k[i]; h *= 0x100000001b3ULL; }
    return h | 1;
}
static void map_init(map_t *m, size_t cap) {
    m->cap = cap; m->n = 0;
    m->s = (slot_t *)calloc(cap, sizeof(slot_t));
    memset(&m->keys, 0, sizeof m->keys);
}
static void map_free(map_t *m) { free(m->s); free(m->keys.p); }
static slot_t *map_find_or_add(map_t *m, const uint8_t *k, size_t len, int *added);
static void map_grow(map_t *m) {
    slot_t *old = m->s;
    size_t oc = m->cap;
    m->cap *= 2;
    m->s = (slot_t *)calloc(m->cap, sizeof(slot_t));
    for (size_t i = 0; i < oc; ++i) {
        if (!old[i].h) continue;
        size_t j = old[i].h & (m->cap - 1);
        while (m->s[j].h) j = (j + 1) & (m->cap - 1);
        m->s[j] = old[i];
    }
    free(old);
}
static slot_t *map_find_or_add(map_t *m, const uint8_t *k, size_t len, int *added) {
    if ((m->n + 1) * 2 > m->cap) map_grow(m);
    uint64_t h = fnv1a(k, len);
    size_t j = h & (m->cap - 1);
    for (;;) {
        slot_t *s = &m->s[j];
        if (!s->h) {
            s->h = h; s->off = m->keys.n; s->len = (uint32_t)len; s->val = 0; s->aux = 0;
            by_put(&m->keys, k, len);
            m->n++;
            *added = 1;
            return s;
        }
        if (s->h == h && s->len == len && !memcmp(m->keys.p + s->off, k, len)) { *added = 0; return s; }
        j = (j + 1) & (m->cap - 1);
    }
}

/* ------------------------------------------------------------------ sorting helpers */

static const uint8_t *g_sort_base;
typedef struct { uint64_t off; uint32_t len; uint32_t part; uint64_t val; uint64_t aux; } ent_t;

static int cmp_bytes(const uint8_t *a, size_t la, const uint8_t *b, size_t lb) {
    size_t l = la < lb ? la : lb;
    int c = memcmp(a, b, l);
    if (c) return c;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}
static int cmp_ent_part_key(const void *x, const void *y) {
    const ent_t *a = (const ent_t *)x, *b = (const ent_t *)y;
    if (a->part != b->part) return a->part < b->part ? -1 : 1;
    return cmp_bytes(g_sort_base + a->off, a->len, g_sort_base + b->off, b->len);
}

/* ------------------------------------------------------------------ FAST wc / indexer */

typedef struct { map_t *m; uint32_t doc; int indexer; } fast_ud;

static void cb_count(void *ud, const uint8_t *k, size_t len) {
    fast_ud *u = (fast_ud *)ud;
    int added;
    slot_t *s = map_find_or_add(u->m, k, len, &added);
    if (!u->indexer) { s->val++; return; }
    /* indexer: aux = bitmap of docs seen would limit docs; keep "last doc" + count of docs, and
     * collect (key, doc) pairs through a second map keyed by key ++ doc. */
    if (added || s->aux != (uint64_t)u->doc + 1) {
        s->aux = (uint64_t)u->doc + 1;   /* docs are visited in order, so this dedups per doc */
        s->val++;
    }
}

/* Emits the reduce output for sorted distinct entries; the last entry of each partition is
 * dropped (worker.rs:169-184 never writes its final group). */
static void emit_sorted(ent_t *e, size_t n, uint32_t R, const uint8_t *keys, bytes_t *out,
                        size_t *part_off, int (*fmt)(void *, const ent_t *, bytes_t *), void *fud) {
    size_t i = 0;
    for (uint32_t r = 0; r < R; ++r) {
        part_off[r] = out->n;
        size_t j = i;
        while (j < n && e[j].part == r) ++j;
        for (size_t t = i; t + 1 < j; ++t) {        /* j-1 is the dropped last group */
            by_put(out, keys + e[t].off, e[t].len);
            by_putc(out, ' ');
            fmt(fud, &e[t], out);
            by_putc(out, '\n');
        }
        i = j;
    }
    part_off[R] = out->n;
}

static int fmt_count(void *ud, const ent_t *e, bytes_t *out) { (void)ud; by_putu64(out, e->val); return 0; }

/* ------------------------------------------------------------------ FAITHFUL wc */

typedef struct { int *fds; uint32_t R; int logfd; int m; int err; } faithful_ud;

static void cb_faithful(void *ud, const uint8_t *k, size_t len) {
    faithful_ud *u = (faithful_ud *)ud;
    uint32_t r = (uint32_t)(oracle_key_hash(k, len) % u->R);             /* worker.rs:129 */
    char line[512];
    char *buf = len + 3 <= sizeof line ? line : (char *)malloc(len + 3);
    memcpy(buf, k, len);
    buf[len] = ' '; buf[len + 1] = '1'; buf[len + 2] = '\n';
    if (write(u->fds[r], buf, len + 3) != (ssize_t)(len + 3)) u->err = 1;  /* :131 one write per token */
    if (buf != line) free(buf);
    char log[160];
    int ll = snprintf(log, sizeof log,                                       /* :132-136 println per token */
                      "[Map] Worker finish mapping task #%d, the intermediate result has been written to mr-%d-%u.txt\n",
                      u->m, u->m, r);
    if (write(u->logfd, log, (size_t)ll) != ll) u->err = 1;
}

typedef struct { const uint8_t *k; uint32_t kl; const uint8_t *v; uint32_t vl; } kv_t;

static int kv_cmp(const kv_t *a, const kv_t *b) { return cmp_bytes(a->k, a->kl, b->k, b->kl); }

static void merge_sort_kv(kv_t *a, kv_t *tmp, size_t n) {   /* stable, like slice::sort_by */
    if (n < 2) return;
    size_t h = n / 2;
    merge_sort_kv(a, tmp, h);
    merge_sort_kv(a + h, tmp, n - h);
    size_t i = 0, j = h, k = 0;
    while (i < h && j < n) tmp[k++] = kv_cmp(&a[j], &a[i]) < 0 ? a[j++] : a[i++];
    while (i < h) tmp[k++] = a[i++];
    while (j < n) tmp[k++] = a[j++];
    memcpy(a, tmp, n * sizeof(kv_t));
}

static int read_all(const char *path, bytes_t *b) {
    int fd = open(path, O_RDONLY);
    if (fd < 0) return ORACLE_EIO;
    struct stat st;
    fstat(fd, &st);
    b->n = 0;
    by_reserve(b, (size_t)st.st_size + 1);
    size_t got = 0;
    while (got < (size_t)st.st_size) {
        ssize_t r = read(fd, b->p + got, (size_t)st.st_size - got);
        if (r <= 0) { close(fd); return ORACLE_EIO; }
        got += (size_t)r;
    }
    b->n = got;
    close(fd);
    return ORACLE_OK;
}

/* One map task (Worker::map, worker.rs:142-155): tokenize file m, one write(2) of "k 1\n" per token to
 * dir/mr-{m}-{r}.txt (r = SipHash % R) and one log line per token. */
static int faithful_map_task(const uint8_t *file, size_t len, int m, uint32_t R, const char *dir, int logfd,
                             bytes_t *scratch) {
    char path[4096];
    int rc = ORACLE_OK;
    int *fds = (int *)malloc(sizeof(int) * R);
    for (uint32_t r = 0; r < R; ++r) {                                       /* :120-125 */
        snprintf(path, sizeof path, "%s/mr-%d-%u.txt", dir, m, r);
        fds[r] = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fds[r] < 0) rc = ORACLE_EIO;
    }
    if (rc == ORACLE_OK) {
        faithful_ud u = {fds, R, logfd, m, 0};
        rc = tokenize(file, len, cb_faithful, &u, scratch);
        if (u.err && rc == ORACLE_OK) rc = ORACLE_EIO;
    }
    for (uint32_t r = 0; r < R; ++r) if (fds[r] >= 0) close(fds[r]);
    free(fds);
    return rc;
}

/* One reduce task (Worker::reduce, worker.rs:157-193): read mr-{m}-{r}.txt for every m, parse, stable
 * sort, group, write dir/mr-{r}.txt; its bytes are also appended to *out. */
static int faithful_reduce_task(int n_files, uint32_t r, const char *dir, bytes_t *out) {
    char path[4096];
    int rc = ORACLE_OK;
    bytes_t all = {0}, content = {0};
    for (int m = 0; m < n_files && rc == ORACLE_OK; ++m) {                   /* read_file_to_mem_reduce :79-109 */
        snprintf(path, sizeof path, "%s/mr-%d-%u.txt", dir, m, r);
        rc = read_all(path, &content);
        if (rc == ORACLE_OK) by_put(&all, content.p, content.n);
    }
    size_t nkv = 0, cap = 1024;
    kv_t *kv = (kv_t *)malloc(sizeof(kv_t) * cap);
    size_t i = 0;
    while (rc == ORACLE_OK && i < all.n) {
        size_t e = i;
        while (e < all.n && all.p[e] != '\n') ++e;
        if (e > i) {
            size_t sp = i;
            while (sp < e && all.p[sp] != ' ') ++sp;
            size_t sp2 = sp + 1;
            while (sp2 < e && all.p[sp2] != ' ') ++sp2;
            if (sp >= e || sp2 != e) { rc = ORACLE_EARG; break; }             /* assert!(len == 2) */
            if (nkv == cap) { cap *= 2; kv = (kv_t *)realloc(kv, sizeof(kv_t) * cap); }
            kv[nkv].k = all.p + i; kv[nkv].kl = (uint32_t)(sp - i);
            kv[nkv].v = all.p + sp + 1; kv[nkv].vl = (uint32_t)(e - sp - 1);
            ++nkv;
        }
        i = e + 1;
    }
    kv_t *tmp = (kv_t *)malloc(sizeof(kv_t) * (nkv ? nkv : 1));
    merge_sort_kv(kv, tmp, nkv);                                             /* :162-164 */
    free(tmp);
    int ofd = -1;
    if (rc == ORACLE_OK) {
        snprintf(path, sizeof path, "%s/mr-%u.txt", dir, r);
        ofd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (ofd < 0) rc = ORACLE_EIO;
    }
    const uint8_t *prev = NULL;
    uint32_t prevl = 0;
    uint64_t nvals = 0;
    for (size_t t = 0; t < nkv && rc == ORACLE_OK; ++t) {                    /* :169-184 */
        if (prevl == 0) { prev = kv[t].k; prevl = kv[t].kl; }            /* :170-172 `prev.is_empty()`: an
                                                                            empty key never stays prev, so empty-key
                                                                            lines fold into the next group */
        if (kv[t].kl != prevl || memcmp(kv[t].k, prev, prevl)) {
            size_t before = out->n;
            by_put(out, prev, prevl);
            by_putc(out, ' ');
            by_putu64(out, nvals);                                           /* wc::reduce */
            by_putc(out, '\n');
            if (write(ofd, out->p + before, out->n - before) != (ssize_t)(out->n - before)) rc = ORACLE_EIO;
            nvals = 0;
            prev = kv[t].k; prevl = kv[t].kl;
        }
        ++nvals;
    }
    /* the final group is never written (no flush after the loop before :185) */
    if (ofd >= 0) close(ofd);
    free(kv); free(all.p); free(content.p);
    return rc;
}

/* The reference job with its own structure, in directory `dir` (intermediates + outputs written
 * there as mr-{m}-{r}.txt / mr-{r}.txt).  Output bytes are also returned concatenated. */
static int wc_faithful(const uint8_t *const *files, const size_t *lens, int n_files, uint32_t R,
                       const char *dir, bytes_t *out, size_t *part_off) {
    int logfd = open("/dev/null", O_WRONLY);
    bytes_t scratch = {0};
    int rc = ORACLE_OK;
    for (int m = 0; m < n_files && rc == ORACLE_OK; ++m) rc = faithful_map_task(files[m], lens[m], m, R, dir, logfd, &scratch);
    for (uint32_t r = 0; r < R && rc == ORACLE_OK; ++r) {
        part_off[r] = out->n;
        rc = faithful_reduce_task(n_files, r, dir, out);
    }
    part_off[R] = out->n;
    free(scratch.p);
    close(logfd);
    return rc;
}

/* ------------------------------------------------------------------ public entry points */

/* Worker::reduce (worker.rs:157-193) on intermediates already in `dir` (mr-{m}-{r}.txt, m < n_files):
 * the bytes of mr-{r}.txt are returned (and written to dir/mr-{r}.txt). */
int oracle_reduce_files(const char *dir, int n_files, uint32_t r, uint8_t **out, size_t *out_len) {
    if (!dir || n_files < 0) return ORACLE_EARG;
    bytes_t o = {0};
    int rc = faithful_reduce_task(n_files, r, dir, &o);
    if (rc != ORACLE_OK) { free(o.p); return rc; }
    *out = o.p ? o.p : (uint8_t *)malloc(1);
    *out_len = o.n;
    return ORACLE_OK;
}

/* Word count over n_files inputs, nReduce = R.  Output: all mr-{r}.txt concatenated in r order
 * (*out, *out_len), with part_off[0..R] byte offsets.  mode ORACLE_FAITHFUL needs `dir`. */
int oracle_wc(const uint8_t *const *files, const size_t *lens, int n_files, uint32_t R, int mode,
              const char *dir, uint8_t **out, size_t *out_len, size_t *part_off) {
    if (R == 0 || n_files < 0) return ORACLE_EARG;
    bytes_t o = {0};
    int rc;
    if (mode == ORACLE_FAITHFUL) {
        if (!dir) return ORACLE_EARG;
        rc = wc_faithful(files, lens, n_files, R, dir, &o, part_off);
    } else {
        map_t m;
        map_init(&m, 1 << 16);
        bytes_t scratch = {0};
        fast_ud u = {&m, 0, 0};
        rc = ORACLE_OK;
        for (int f = 0; f < n_files && rc == ORACLE_OK; ++f) rc = tokenize(files[f], lens[f], cb_count, &u, &scratch);
        free(scratch.p);
        if (rc == ORACLE_OK) {
            ent_t *e = (ent_t *)malloc(sizeof(ent_t) * (m.n ? m.n : 1));
            size_t k = 0;
            for (size_t i = 0; i < m.cap; ++i) {
                if (!m.s[i].h) continue;
                e[k].off = m.s[i].off; e[k].len = m.s[i].len; e[k].val = m.s[i].val; e[k].aux = 0;
                e[k].part = (uint32_t)(oracle_key_hash(m.keys.p + m.s[i].off, m.s[i].len) % R);
                ++k;
            }
            g_sort_base = m.keys.p;
            qsort(e, k, sizeof(ent_t), cmp_ent_part_key);
            emit_sorted(e, k, R, m.keys.p, &o, part_off, fmt_count, NULL);
            free(e);
        }
        map_free(&m);
    }
    if (rc) { free(o.p); return rc; }
    *out = o.p ? o.p : (uint8_t *)malloc(1);
    *out_len = o.n;
    return ORACLE_OK;
}

/* ---- indexer (build-defined app; no indexer exists in the reference) ----
 * map(doc, text) emits (word, doc) once per distinct word of a document; reduce(word, docs)
 * returns "{n} {docs sorted bytewise, comma-joined}"; same worker loop (drop-last included). */

typedef struct { map_t *words; map_t *pairs; uint32_t doc; bytes_t *tmp; } idx_ud;

static void cb_index(void *ud, const uint8_t *k, size_t len) {
    idx_ud *u = (idx_ud *)ud;
    int added;
    slot_t *s = map_find_or_add(u->words, k, len, &added);
    if (s->aux == (uint64_t)u->doc + 1) return;     /* already emitted for this document */
    s->aux = (uint64_t)u->doc + 1;
    s->val++;
    /* record the pair under key "word\0<doc>" (keys never contain NUL) */
    u->tmp->n = 0;
    by_put(u->tmp, k, len);
    by_putc(u->tmp, 0);
    by_put(u->tmp, &u->doc, sizeof u->doc);
    map_find_or_add(u->pairs, u->tmp->p, u->tmp->n, &added);
}

typedef struct { const char *const *docs; const uint32_t *rank; uint32_t n_docs; uint32_t **lists; } idx_fmt_ud;

static const uint32_t *g_rank;
static int cmp_doc_by_rank(const void *a, const void *b) {
    uint32_t x = g_rank[*(const uint32_t *)a], y = g_rank[*(const uint32_t *)b];
    return x < y ? -1 : (x > y ? 1 : 0);
}

static int fmt_index(void *ud, const ent_t *e, bytes_t *out) {
    idx_fmt_ud *f = (idx_fmt_ud *)ud;
    uint32_t *list = f->lists[e->aux];
    uint32_t n = list[0];
    g_rank = f->rank;
    qsort(list + 1, n, sizeof(uint32_t), cmp_doc_by_rank);
    by_putu64(out, n);
    by_putc(out, ' ');
    for (uint32_t i = 0; i < n; ++i) {
        if (i) by_putc(out, ',');
        const char *d = f->docs[list[1 + i]];
        by_put(out, d, strlen(d));
    }
    return 0;
}

static const char *const *g_docs;
static int cmp_doc_names(const void *a, const void *b) {
    const char *x = g_docs[*(const uint32_t *)a], *y = g_docs[*(const uint32_t *)b];
    return cmp_bytes((const uint8_t *)x, strlen(x), (const uint8_t *)y, strlen(y));
}

int oracle_indexer(const uint8_t *const *files, const size_t *lens, const char *const *docs, int n_files,
                   uint32_t R, uint8_t **out, size_t *out_len, size_t *part_off) {
    if (R == 0 || n_files < 0) return ORACLE_EARG;
    for (int i = 0; i < n_files; ++i)
        for (const char *c = docs[i]; *c; ++c)
            if (*c == ' ' || *c == '\n' || *c == ',') return ORACLE_EARG;   /* worker.rs:100 2-field parse */
    map_t words, pairs;
    map_init(&words, 1 << 16);
    map_init(&pairs, 1 << 16);
    bytes_t scratch = {0}, tmp = {0};
    int rc = ORACLE_OK;
    for (int f = 0; f < n_files && rc == ORACLE_OK; ++f) {
        idx_ud u = {&words, &pairs, (uint32_t)f, &tmp};
        rc = tokenize(files[f], lens[f], cb_index, &u, &scratch);
    }
    free(scratch.p); free(tmp.p);
    bytes_t o = {0};
    if (rc == ORACLE_OK) {
        /* doc lists per word */
        size_t nw = words.n;
        ent_t *e = (ent_t *)malloc(sizeof(ent_t) * (nw ? nw : 1));
        uint32_t **lists = (uint32_t **)malloc(sizeof(uint32_t *) * (nw ? nw : 1));
        size_t k = 0;
        for (size_t i = 0; i < words.cap; ++i) {
            if (!words.s[i].h) continue;
            e[k].off = words.s[i].off; e[k].len = words.s[i].len; e[k].val = words.s[i].val;
            e[k].aux = k;
            e[k].part = (uint32_t)(oracle_key_hash(words.keys.p + words.s[i].off, words.s[i].len) % R);
            lists[k] = (uint32_t *)malloc(sizeof(uint32_t) * (words.s[i].val + 1));
            lists[k][0] = 0;
            words.s[i].aux = k;   /* reuse aux as list id */
            ++k;
        }
        for (size_t i = 0; i < pairs.cap; ++i) {
            if (!pairs.s[i].h) continue;
            const uint8_t *pk = pairs.keys.p + pairs.s[i].off;
            size_t wl = pairs.s[i].len - 1 - sizeof(uint32_t);
            uint32_t doc;
            memcpy(&doc, pk + wl + 1, sizeof doc);
            int added;
            slot_t *w = map_find_or_add(&words, pk, wl, &added);
            uint32_t *l = lists[w->aux];
            l[1 + l[0]++] = doc;
        }
        uint32_t *order = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n_files ? n_files : 1));
        uint32_t *rank = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n_files ? n_files : 1));
        for (int i = 0; i < n_files; ++i) order[i] = (uint32_t)i;
        g_docs = docs;
        qsort(order, (size_t)n_files, sizeof(uint32_t), cmp_doc_names);
        for (int i = 0; i < n_files; ++i) rank[order[i]] = (uint32_t)i;
        g_sort_base = words.keys.p;
        qsort(e, k, sizeof(ent_t), cmp_ent_part_key);
        idx_fmt_ud fu = {docs, rank, (uint32_t)n_files, lists};
        emit_sorted(e, k, R, words.keys.p, &o, part_off, fmt_index, &fu);
        for (size_t i = 0; i < k; ++i) free(lists[i]);
        free(lists); free(e); free(order); free(rank);
    }
    map_free(&words); map_free(&pairs);
    if (rc) { free(o.p); return rc; }
    *out = o.p ? o.p : (uint8_t *)malloc(1);
    *out_len = o.n;
    return ORACLE_OK;
}

/* ------------------------------------------------------------------ W worker threads (FAITHFUL) */

/* The reference's process structure (mrworker.rs:43-149): W workers pull map task ids from the
 * coordinator (coordinator.rs:137-176), then -- after every map task is done -- reduce task ids
 * (:178-215).  Threads here, processes there; each task is the single-threaded FAITHFUL task. */
typedef struct {
    const uint8_t *const *files; const size_t *lens; int n_files; uint32_t R; const char *dir;
    int next_map, next_reduce, rc; bytes_t *outs; pthread_mutex_t mu; pthread_barrier_t maps_done;
} workers_t;

static int take(workers_t *w, int *next, int limit) {
    pthread_mutex_lock(&w->mu);
    int t = (w->rc == ORACLE_OK && *next < limit) ? (*next)++ : -1;
    pthread_mutex_unlock(&w->mu);
    return t;
}
static void fail(workers_t *w, int rc) {
    pthread_mutex_lock(&w->mu);
    if (w->rc == ORACLE_OK) w->rc = rc;
    pthread_mutex_unlock(&w->mu);
}

static void *worker_main(void *arg) {
    workers_t *w = (workers_t *)arg;
    int logfd = open("/dev/null", O_WRONLY);
    bytes_t scratch = {0};
    for (int m; (m = take(w, &w->next_map, w->n_files)) >= 0;) {
        int rc = faithful_map_task(w->files[m], w->lens[m], m, w->R, w->dir, logfd, &scratch);
        if (rc) fail(w, rc);
    }
    pthread_barrier_wait(&w->maps_done);   /* the coordinator's phase barrier (map_finish) */
    for (int r; (r = take(w, &w->next_reduce, (int)w->R)) >= 0;) {
        int rc = faithful_reduce_task(w->n_files, (uint32_t)r, w->dir, &w->outs[r]);
        if (rc) fail(w, rc);
    }
    free(scratch.p);
    close(logfd);
    return NULL;
}

int oracle_wc_workers(const uint8_t *const *files, const size_t *lens, int n_files, uint32_t R, int W,
                      const char *dir, uint8_t **out, size_t *out_len, size_t *part_off) {
    if (R == 0 || n_files < 0 || W < 1 || !dir) return ORACLE_EARG;
    workers_t w;
    memset(&w, 0, sizeof w);
    w.files = files; w.lens = lens; w.n_files = n_files; w.R = R; w.dir = dir; w.rc = ORACLE_OK;
    w.outs = (bytes_t *)calloc(R, sizeof(bytes_t));
    pthread_mutex_init(&w.mu, NULL);
    pthread_barrier_init(&w.maps_done, NULL, (unsigned)W);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)W);
    for (int i = 0; i < W; ++i) pthread_create(&th[i], NULL, worker_main, &w);
    for (int i = 0; i < W; ++i) pthread_join(th[i], NULL);
    free(th);
    pthread_barrier_destroy(&w.maps_done);
    pthread_mutex_destroy(&w.mu);
    bytes_t o = {0};
    for (uint32_t r = 0; r < R; ++r) {
        part_off[r] = o.n;
        if (w.outs[r].n) by_put(&o, w.outs[r].p, w.outs[r].n);
        free(w.outs[r].p);
    }
    part_off[R] = o.n;
    free(w.outs);
    if (w.rc) { free(o.p); return w.rc; }
    *out = o.p ? o.p : (uint8_t *)malloc(1);
    *out_len = o.n;
    return ORACLE_OK;
}

/* ------------------------------------------------------------------ FAST on T threads */

/* The input is cut into chunks at ASCII White_Space bytes (a token never spans one; UTF-8 never
 * has a byte < 0x80 inside a multi-byte sequence), each thread counts its chunks into NSUB sub-maps
 * chosen by the key's FNV hash, then sub-map p of every thread is merged by one thread, partitioned
 * by SipHash % R, and every partition is sorted and written by one thread.  Output = oracle_wc FAST. */
#define MT_NSUB 64
typedef struct { const uint8_t *p; size_t n; } chunk_t;
typedef struct { const uint8_t *k; uint32_t len; uint32_t part; uint64_t val; } kent_t;

typedef struct {
    chunk_t *chunks; size_t n_chunks; int T; uint32_t R;
    map_t *sub;              /* [T][NSUB] */
    kent_t **ents; size_t *n_ents;   /* per sub-map after the merge */
    size_t **pcount;         /* [NSUB][R] entries of sub p in partition r */
    bytes_t *outs;           /* per partition */
    int next, rc; pthread_mutex_t mu; pthread_barrier_t bar;
} mt_t;

typedef struct { mt_t *g; int t; } mt_arg;
typedef struct { map_t *sub; } mt_ud;

static void cb_count_mt(void *ud, const uint8_t *k, size_t len) {
    mt_ud *u = (mt_ud *)ud;
    uint64_t h = fnv1a(k, len);
    int added;
    slot_t *s = map_find_or_add(&u->sub[h >> 58], k, len, &added);
    s->val++;
}

static int mt_take(mt_t *g, int limit) {
    pthread_mutex_lock(&g->mu);
    int t = g->next < limit ? g->next++ : -1;
    pthread_mutex_unlock(&g->mu);
    return t;
}

static int cmp_kent(const void *x, const void *y) {
    const kent_t *a = (const kent_t *)x, *b = (const kent_t *)y;
    return cmp_bytes(a->k, a->len, b->k, b->len);
}

#include <time.h>
static double now_s(void) { struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); return ts.tv_sec + 1e-9 * ts.tv_nsec; }
static void *mt_main(void *arg) {
    mt_arg *a = (mt_arg *)arg;
    const int dbg = getenv("ORACLE_MT_DEBUG") != NULL;
    double t0 = now_s();
    mt_t *g = a->g;
    const int t = a->t;
    map_t *mine = &g->sub[(size_t)t * MT_NSUB];
    bytes_t scratch = {0};
    mt_ud u = {mine};
    for (int c; (c = mt_take(g, (int)g->n_chunks)) >= 0;) {
        int rc = tokenize(g->chunks[c].p, g->chunks[c].n, cb_count_mt, &u, &scratch);
        if (rc) { pthread_mutex_lock(&g->mu); g->rc = rc; pthread_mutex_unlock(&g->mu); }
    }
    free(scratch.p);
    if (dbg) fprintf(stderr, "t%d count %.3f\n", t, now_s() - t0);
    if (pthread_barrier_wait(&g->bar) == PTHREAD_BARRIER_SERIAL_THREAD) g->next = 0;
    pthread_barrier_wait(&g->bar);
    if (dbg && t == 0) fprintf(stderr, "barrier1 %.3f\n", now_s() - t0);
    /* merge sub-map p of every thread into thread 0's, then list its entries with their partition */
    for (int p; (p = mt_take(g, MT_NSUB)) >= 0;) {
        map_t *dst = &g->sub[p];
        for (int o = 1; o < g->T; ++o) {
            map_t *src = &g->sub[(size_t)o * MT_NSUB + p];
            for (size_t i = 0; i < src->cap; ++i) {
                if (!src->s[i].h) continue;
                int added;
                slot_t *d = map_find_or_add(dst, src->keys.p + src->s[i].off, src->s[i].len, &added);
                d->val += src->s[i].val;
            }
            map_free(src);
            memset(src, 0, sizeof *src);
        }
        kent_t *e = (kent_t *)malloc(sizeof(kent_t) * (dst->n ? dst->n : 1));
        size_t k = 0;
        g->pcount[p] = (size_t *)calloc(g->R, sizeof(size_t));
        for (size_t i = 0; i < dst->cap; ++i) {
            if (!dst->s[i].h) continue;
            e[k].k = dst->keys.p + dst->s[i].off;
            e[k].len = dst->s[i].len;
            e[k].val = dst->s[i].val;
            e[k].part = (uint32_t)(oracle_key_hash(e[k].k, e[k].len) % g->R);
            g->pcount[p][e[k].part]++;
            ++k;
        }
        g->ents[p] = e;
        g->n_ents[p] = k;
    }
    if (pthread_barrier_wait(&g->bar) == PTHREAD_BARRIER_SERIAL_THREAD) g->next = 0;
    pthread_barrier_wait(&g->bar);
    if (dbg && t == 0) fprintf(stderr, "barrier2 %.3f\n", now_s() - t0);
    /* partition r: gather, sort by key bytes, format, drop the last group */
    for (int r; (r = mt_take(g, (int)g->R)) >= 0;) {
        size_t n = 0;
        for (int p = 0; p < MT_NSUB; ++p) n += g->pcount[p][r];
        kent_t *e = (kent_t *)malloc(sizeof(kent_t) * (n ? n : 1));
        size_t k = 0;
        for (int p = 0; p < MT_NSUB; ++p)
            for (size_t i = 0; i < g->n_ents[p]; ++i)
                if (g->ents[p][i].part == (uint32_t)r) e[k++] = g->ents[p][i];
        qsort(e, k, sizeof(kent_t), cmp_kent);
        bytes_t *o = &g->outs[r];
        for (size_t i = 0; i + 1 < k; ++i) {   /* worker.rs:169-184: the last group is never written */
            by_put(o, e[i].k, e[i].len);
            by_putc(o, ' ');
            by_putu64(o, e[i].val);
            by_putc(o, '\n');
        }
        free(e);
    }
    return NULL;
}

int oracle_wc_mt(const uint8_t *const *files, const size_t *lens, int n_files, uint32_t R, int T,
                 uint8_t **out, size_t *out_len, size_t *part_off) {
    if (R == 0 || n_files < 0 || T < 1) return ORACLE_EARG;
    size_t total = 0;
    for (int f = 0; f < n_files; ++f) total += lens[f];
    const size_t target = total / ((size_t)T * 8) + (1u << 20);
    size_t cap = 16, nc = 0;
    chunk_t *ch = (chunk_t *)malloc(sizeof(chunk_t) * cap);
    for (int f = 0; f < n_files; ++f) {
        const uint8_t *s = files[f];
        size_t a = 0;
        while (a < lens[f]) {
            size_t b = a + target < lens[f] ? a + target : lens[f];
            while (b < lens[f] && !(s[b] == ' ' || (s[b] >= 0x09 && s[b] <= 0x0D))) ++b;
            if (nc == cap) { cap *= 2; ch = (chunk_t *)realloc(ch, sizeof(chunk_t) * cap); }
            ch[nc].p = s + a;
            ch[nc].n = b - a;
            ++nc;
            a = b;
        }
    }
    mt_t g;
    memset(&g, 0, sizeof g);
    g.chunks = ch; g.n_chunks = nc; g.T = T; g.R = R;
    g.sub = (map_t *)calloc((size_t)T * MT_NSUB, sizeof(map_t));
    for (size_t i = 0; i < (size_t)T * MT_NSUB; ++i) map_init(&g.sub[i], 1 << 10);
    g.ents = (kent_t **)calloc(MT_NSUB, sizeof(kent_t *));
    g.n_ents = (size_t *)calloc(MT_NSUB, sizeof(size_t));
    g.pcount = (size_t **)calloc(MT_NSUB, sizeof(size_t *));
    g.outs = (bytes_t *)calloc(R, sizeof(bytes_t));
    pthread_mutex_init(&g.mu, NULL);
    pthread_barrier_init(&g.bar, NULL, (unsigned)T);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)T);
    mt_arg *args = (mt_arg *)malloc(sizeof(mt_arg) * (size_t)T);
    for (int t = 0; t < T; ++t) {
        args[t].g = &g;
        args[t].t = t;
        pthread_create(&th[t], NULL, mt_main, &args[t]);
    }
    for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
    bytes_t o = {0};
    for (uint32_t r = 0; r < R; ++r) {
        part_off[r] = o.n;
        if (g.outs[r].n) by_put(&o, g.outs[r].p, g.outs[r].n);
        free(g.outs[r].p);
    }
    part_off[R] = o.n;
    for (size_t i = 0; i < (size_t)T * MT_NSUB; ++i) map_free(&g.sub[i]);
    for (int p = 0; p < MT_NSUB; ++p) { free(g.ents[p]); free(g.pcount[p]); }
    free(g.sub); free(g.ents); free(g.n_ents); free(g.pcount); free(g.outs); free(th); free(args); free(ch);
    pthread_barrier_destroy(&g.bar);
    pthread_mutex_destroy(&g.mu);
    if (g.rc) { free(o.p); return g.rc; }
    *out = o.p ? o.p : (uint8_t *)malloc(1);
    *out_len = o.n;
    return ORACLE_OK;
}

void oracle_free(void *p) { free(p); }
