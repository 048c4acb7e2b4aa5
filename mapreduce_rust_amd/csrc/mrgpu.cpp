// mrgpu.cpp -- C ABI (include/mrgpu.h) and host orchestration of libmrgpu.so.
//
// Pipeline of one job, all on one HIP stream of the context:
//   map     k_map (tokenize + LDS combine)                         wc.rs:6-13, worker.rs:117-131
//   agg     HBM table insert/compact + long-key fingerprint sort   worker.rs:165-184 (grouping)
//           + SipHash-1-3 % R per distinct key                     worker.rs:111-115, 129
//   [shuffle: export by owner = r % G, exchange by the caller (RCCL all-to-all), import]
//   reduce  radix sort by (r, key bytes[, doc]) + format lines     worker.rs:162-184, wc.rs:15-17
// Errors never cross the ABI as exceptions or aborts: every entry point returns a status code.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>

#include <rccl/rccl.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mrg_internal.h"
#include "mrgpu.h"

static_assert(sizeof(XRec) == MRG_XREC_BYTES, "exchange record layout (include/mrgpu.h)");

namespace {

thread_local std::string g_err;

struct MrgError {
    int code;
    std::string msg;
};

[[noreturn]] void raise(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw MrgError{code, buf};
}

#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) raise(MRG_EHIP, "%s: %s", #x, hipGetErrorString(e_));    \
    } while (0)

#define NCCLCHK(x)                                                                     \
    do {                                                                               \
        ncclResult_t r_ = (x);                                                         \
        if (r_ != ncclSuccess) raise(MRG_ECOMM, "%s: %s", #x, ncclGetErrorString(r_)); \
    } while (0)

// The radix sorts index records with 32-bit offsets (k_sort.hip): refuse larger inputs loudly.
void check_sort_n(uint64_t n, const char *what) {
    if (n > 0xFFFFFFFFull) raise(MRG_ENOMEM, "%s: %llu records exceed the radix sort's 32-bit index", what,
                                 (unsigned long long)n);
}

// Test knobs (env, read once per map): shrink the map's tail regions and overflow lists on the first
// launch so the spill and grow-and-rerun paths run on small inputs.
uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *v = getenv(name);
    return v && *v ? strtoull(v, nullptr, 10) : dflt;
}
// MRG_WIDE=<non-zero>: force the wide (sort-based) aggregation; MRG_WIDE=0 pins the bucket path
bool wide_forced() {
    const char *v = getenv("MRG_WIDE");
    return v && *v && atoi(v) != 0;
}
// MRG_WIDE=0 pins the bucket path, so it also rules out the wide map
bool wide_forced_off() {
    const char *v = getenv("MRG_WIDE");
    return v && *v && atoi(v) == 0;
}

template <class F>
int guard(F &&f) {
    try {
        f();
        return MRG_OK;
    } catch (const MrgError &e) {
        g_err = e.msg;
        return e.code;
    } catch (const std::bad_alloc &) {
        g_err = "host out of memory";
        return MRG_ENOMEM;
    } catch (...) {
        g_err = "unexpected internal error";
        return MRG_EINVAL;
    }
}

// ---------------------------------------------------------------- caching device allocator
// Process-wide cache of the device blocks of closed contexts, per device (r06).  A worker process runs
// one task after another (src/bin/mrworker.rs:43-149); every mrg_run_job opens fresh contexts, and
// without this each call re-allocated -- and the GPU re-touched -- its multi-GiB workspaces (the first
// job's map ran 1.2x its steady time).  Capped at MRG_POOL_KEEP_GIB per device (default: half the
// device's memory; 0 = off); blocks beyond the cap are freed.  Never destroyed: no hipFree may run
// after the HIP runtime's own teardown at process exit.
class DeviceCache {
   public:
    static DeviceCache &get() {
        static DeviceCache *c = new DeviceCache();
        return *c;
    }
    // a cached block of `dev` of at least c bytes and at most c + c / 4 (any size >= c when `any`: the
    // device is full) -- its size in *got -- else null
    void *take(int dev, size_t c, size_t *got, bool any = false) {
        std::lock_guard<std::mutex> lk(mu_);
        auto &f = free_[dev];
        auto it = f.lower_bound(c);
        if (it == f.end() || (!any && it->first > c + (c >> 2))) return nullptr;
        void *p = it->second;
        *got = it->first;
        bytes_[dev] -= it->first;
        f.erase(it);
        return p;
    }
    // a block of a closing context (its work on the device finished); the current device is `dev`
    void give(int dev, void *p, size_t c) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (bytes_[dev] + c <= keep(dev)) {
                free_[dev].insert({c, p});
                bytes_[dev] += c;
                return;
            }
        }
        (void)hipFree(p);
    }
    void trim(int dev) {  // the device is full: give the cached blocks back to the driver
        std::multimap<size_t, void *> f;
        {
            std::lock_guard<std::mutex> lk(mu_);
            f.swap(free_[dev]);
            bytes_[dev] = 0;
        }
        for (auto &kv : f) (void)hipFree(kv.second);
    }

   private:
    DeviceCache() {
        if (const char *v = getenv("MRG_POOL_KEEP_GIB")) keep_env_ = (long long)(atof(v) * (double)((size_t)1 << 30));
    }
    // bytes of `dev` (the current device) kept: MRG_POOL_KEEP_GIB, else half the device's memory.  A
    // block handed back to the driver is wiped before any allocation can reuse it (a fresh context
    // after one that freed ~100 GiB waited 4.6 s in hipMalloc: profiles/r06/v13), so one C5-sized
    // job's blocks (67-83 GiB at 13.4 GB of input) are worth keeping
    size_t keep(int dev) {
        if (keep_env_ >= 0) return (size_t)keep_env_;
        auto it = keep_dev_.find(dev);
        if (it != keep_dev_.end()) return it->second;
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
            (void)hipGetLastError();
            tot = (size_t)128 << 30;
        }
        return keep_dev_[dev] = tot / 2;
    }
    std::mutex mu_;
    std::map<int, std::multimap<size_t, void *>> free_;
    std::map<int, size_t> bytes_;
    std::map<int, size_t> keep_dev_;
    long long keep_env_ = -1;
};

class Pool : public DevPool {
   public:
    void set_device(int dev) { dev_ = dev; }
    void *get(size_t bytes) override {
        const size_t c = cls(bytes ? bytes : 1);
        // smallest free block of this class or up to two classes above (record counts drift by a few
        // between jobs over the same input: an exact-class pool would then miss, run out of device
        // memory and trim everything)
        auto it = free_.lower_bound(c);
        if (it != free_.end() && it->first <= c + (c >> 2)) {
            void *p = it->second;
            free_.erase(it);
            return p;
        }
        if (dev_ >= 0) {  // a block a closed context of this device left behind
            size_t got = 0;
            if (void *q = DeviceCache::get().take(dev_, c, &got)) {
                size_[q] = got;
                ++reused_;
                return q;
            }
        }
        void *p = nullptr;
        if (debug_) fprintf(stderr, "[mrgpu] pool: allocating %zu bytes\n", c);
        const auto t0 = std::chrono::steady_clock::now();
        if (hipMalloc(&p, c) != hipSuccess) {
            (void)hipGetLastError();
            // the device is full: a larger cached block first (memory handed back to the driver is
            // wiped before it can be allocated again: a trim costs seconds)
            if (dev_ >= 0) {
                size_t got = 0;
                if (void *q = DeviceCache::get().take(dev_, c, &got, true)) {
                    alloc_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                    size_[q] = got;
                    ++reused_;
                    return q;
                }
            }
            if (debug_) fprintf(stderr, "[mrgpu] pool: device full, trimming %zu free blocks\n", free_.size());
            trim();
            if (hipMalloc(&p, c) != hipSuccess) {
                (void)hipGetLastError();
                raise(MRG_ENOMEM, "device allocation of %zu bytes failed", c);
            }
        }
        alloc_ms_ += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        ++allocs_;
        alloc_bytes_ += c;
        size_[p] = c;
        return p;
    }
    void put(void *p) override {
        if (!p) return;
        auto it = size_.find(p);
        if (it != size_.end()) free_.insert({it->second, p});
    }
    void trim() {
        (void)hipDeviceSynchronize();
        for (auto &kv : free_) {
            (void)hipFree(kv.second);
            size_.erase(kv.second);
        }
        free_.clear();
        if (dev_ >= 0) DeviceCache::get().trim(dev_);
    }
    // blocks handed out and not returned; bytes held by the pool (handed out or cached)
    uint64_t outstanding() const { return size_.size() - free_.size(); }
    uint64_t held_bytes() const {
        uint64_t b = 0;
        for (auto &kv : size_) b += kv.second;
        return b;
    }
    // device allocations made so far (hipMalloc calls, bytes, host milliseconds inside them): a fresh
    // context's first job pays them, later jobs reuse the cached blocks
    void alloc_stats(uint64_t *n, uint64_t *bytes, double *ms) const {
        if (n) *n = allocs_;
        if (bytes) *bytes = alloc_bytes_;
        if (ms) *ms = alloc_ms_;
    }
    uint64_t reused() const { return reused_; }  // blocks taken from the process-wide device cache
    ~Pool() override {  // (the caller has made dev_ current)
        (void)hipDeviceSynchronize();
        for (auto &kv : size_) {
            if (dev_ >= 0) DeviceCache::get().give(dev_, kv.first, kv.second);
            else (void)hipFree(kv.first);
        }
    }

   private:
    static size_t cls(size_t b) {
        if (b <= 4096) return (b + 255) & ~(size_t)255;
        size_t p = 4096;
        while (p < b) p <<= 1;
        const size_t step = p >> 3;  // 8 classes per octave: <= 12.5% slack
        return ((b + step - 1) / step) * step;
    }
    std::multimap<size_t, void *> free_;
    std::unordered_map<void *, size_t> size_;
    bool debug_ = getenv("MRG_DEBUG") != nullptr;
    uint64_t allocs_ = 0, alloc_bytes_ = 0, reused_ = 0;
    int dev_ = -1;
    double alloc_ms_ = 0.0;
};

template <class T>
T *pget(Pool &p, uint64_t n) {
    return (T *)p.get(sizeof(T) * (n ? n : 1));
}

struct KeysBuf {
    KeySet ks{};
    uint64_t n = 0, cap = 0;
    uint8_t *heap = nullptr;
    uint64_t heap_bytes = 0;
    bool any_long = false;
    bool sorted = false;  // keys already in (partition, key) order (wide aggregation, no long keys)
};

// Result of the wide (sample-sort) aggregation, k_wide.hip: distinct keys in output order, per leaf,
// with gaps between leaves; formatted directly, or made a dense KeySet for the other consumers.
struct WideRes {
    bool ready = false;
    uint32_t B1 = 0, B1r = 0;
    uint64_t *kout = nullptr, *ocnt = nullptr;
    uint32_t *nleaf = nullptr, *leaf_nd = nullptr, *leaf_last = nullptr, *leaf_pk = nullptr;
    uint64_t *leaf_out = nullptr, *leaf_bytes = nullptr;
    uint64_t distinct = 0;
    void release(Pool &p) {
        p.put(kout); p.put(ocnt); p.put(nleaf); p.put(leaf_nd); p.put(leaf_last); p.put(leaf_out); p.put(leaf_bytes);
        p.put(leaf_pk);
        *this = WideRes{};
    }
};

}  // namespace

struct mrg_ctx {
    int device = 0;
    hipStream_t own = nullptr, stream = nullptr;
    Pool pool;
    unsigned long long *d_cnt = nullptr;  // CNT_N counters
    unsigned long long *h_cnt = nullptr;  // pinned mirror
    // pinned staging of the small per-job host tables (document offsets, region bases, map args): one
    // bump region, reset by job_begin (after its sync), so their copies are plain async DMA
    uint8_t *h_stage = nullptr;
    size_t stage_used = 0;
    // batched small writes (stage_h2d / stage_fill): their device copy of the staging buffer, the ops
    // not yet issued, and the first staging byte they use
    uint8_t *d_stage = nullptr;
    std::vector<StageOp> pend;
    size_t pend_lo = 0;
    bool timing = false;
    hipEvent_t ev[8] = {};
    int lds_cap = 4096;
    int map_grid = 0;
    uint64_t long_hint = 0, ovf_hint = 0;
    uint64_t lper_hint = 0;  // long-token records per map workgroup region (grown on a rerun)
    uint32_t agg_nsub = 1;  // bucket-aggregation workgroups per bucket (grown when the tables overflow)
    std::vector<double> bcap_rate;  // tail records per (bucket, map workgroup) per input byte of the workgroup
    std::vector<double> bcap16_rate;  // the same for the 16-byte regions (wc keys of 13..16 bytes)
    uint64_t ocap_hint = 0;         // records per bucket overflow list
    bool spec_agg = false, spec_c32 = false;  // last wc job took the bucket path (with 32-bit counts)
    bool wide_hint = false;   // last wc job took the wide aggregation (the next one may take the wide map)
    bool wc_sized = false;    // a wc job of >= 64 MiB has run on this context (its path is a measured hint)
    uint64_t wcap_hint = 0;   // wide map: records per (L1 bucket, workgroup) region the last run needed
    bool w12_off = false;     // wide map: a job overflowed the 16-byte lists of the 12-byte regions
    // job
    bool job = false;
    int app = 0;
    uint32_t R = 0, flags = 0;
    const uint8_t *d_in = nullptr;
    std::vector<uint64_t> doc_off;
    std::vector<uint32_t> doc_ids;
    std::vector<std::string> names;
    KeysBuf keys;
    WideRes wide;
    bool mapped = false;
    uint32_t n_owners = 0;
    std::vector<uint64_t> exp_rec, exp_heap;
    uint64_t xrec_vmax = MRG_XREC_VMAX;  // count per short export record (test knob MRG_TEST_XREC_VMAX)
    uint8_t *d_out = nullptr;
    uint64_t out_cap = 0, out_bytes = 0;
    std::vector<uint64_t> part_off;
    bool reduced = false;
    uint8_t *d_final = nullptr;     // final.txt (mrg_job_final)
    uint64_t final_cap = 0, final_bytes = 0;
    bool finalized = false;
    uint64_t extra_first = 0;       // text reduce: values of empty-key lines, folded into the first group
    mrg_stats st{};
};

struct mrg_comm {
    ncclComm_t comm = nullptr;
    int n = 0, rank = 0, device = 0;
    // preallocated at init, so the exchange never allocates before a collective that its peers are
    // already waiting in: the counts message [3 * n send | 3 * n receive] and the status word
    uint64_t *d_counts = nullptr;
    int *d_flag = nullptr;
    std::atomic<bool> aborted{false};  // ncclCommAbort was called (by this rank or by mrg_run_job's watchdog)
    // held around every RCCL enqueue of a rank thread and around the abort, so mrg_run_job's watchdog
    // does not free the communicator (ncclCommAbort) between a rank thread's aborted-check and its
    // RCCL call; never held across a wait on the stream
    std::timed_mutex mu;
};

struct mrg_parts {
    uint32_t R = 0;
    std::vector<uint64_t> rec_off, heap_off;  // [R + 1]
    std::vector<uint8_t> recs, heap;
};

namespace {

uint32_t hash_bits(const mrg_ctx *c) { return (c->flags >> 8) & 0xFFu; }
bool is_idx(const mrg_ctx *c) { return c->app == MRG_APP_INDEXER; }

void sync(mrg_ctx *c) { HIPCHK(hipStreamSynchronize(c->stream)); }

constexpr size_t MRG_STAGE_BYTES = 256u << 10;
// Host -> device copy of a small table through the pinned staging region (falls back to a pageable
// copy when the region is used up).  Valid only between job_begin and the job's next host wait.
void h2d(mrg_ctx *c, void *dst, const void *src, size_t n) {
    if (!n) return;
    if (c->h_stage && c->stage_used + n <= MRG_STAGE_BYTES) {
        uint8_t *p = c->h_stage + c->stage_used;
        memcpy(p, src, n);
        c->stage_used += (n + 63) & ~(size_t)63;
        HIPCHK(hipMemcpyAsync(dst, p, n, hipMemcpyHostToDevice, c->stream));
    } else {
        HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->stream));
    }
}

// Batched small writes of a job's setup (r06): data staged in the pinned buffer like h2d's, the writes
// recorded, and issued together by flush_stage -- one copy of the staged range (ops table included)
// and one k_stage_scatter launch instead of a copy or memset each (C3 map setup: 12 -> 2 stream ops).
// Every kernel that reads a staged destination must be launched after a flush_stage.
constexpr size_t MRG_STAGE_OPS = 256;   // ops per batch
constexpr uint32_t MRG_STAGE_MAX = 16384;  // larger writes go through their own copy / memset
void flush_stage(mrg_ctx *c) {
    if (c->pend.empty()) return;
    const size_t t = (c->stage_used + 63) & ~(size_t)63;  // the ops table after the staged data
    const size_t tb = sizeof(StageOp) * c->pend.size();
    memcpy(c->h_stage + t, c->pend.data(), tb);
    HIPCHK(hipMemcpyAsync(c->d_stage + c->pend_lo, c->h_stage + c->pend_lo, t + tb - c->pend_lo, hipMemcpyHostToDevice,
                          c->stream));
    mrg_launch_stage_scatter(c->d_stage, (uint32_t)t, (uint32_t)c->pend.size(), c->stream);
    HIPCHK(hipGetLastError());
    c->stage_used = c->pend_lo = (t + tb + 63) & ~(size_t)63;
    c->pend.clear();
}
bool stage_room(mrg_ctx *c, size_t n) {
    if (!c->h_stage || !c->d_stage || n > MRG_STAGE_MAX) return false;
    if (c->pend.size() >= MRG_STAGE_OPS ||
        c->stage_used + n + 64 + sizeof(StageOp) * (MRG_STAGE_OPS + 1) > MRG_STAGE_BYTES) {
        flush_stage(c);
        if (c->stage_used + n + 64 + sizeof(StageOp) * (MRG_STAGE_OPS + 1) > MRG_STAGE_BYTES) return false;
    }
    return true;
}
void stage_h2d(mrg_ctx *c, void *dst, const void *src, size_t n) {
    if (!n) return;
    if (!stage_room(c, n)) {
        flush_stage(c);  // (issue order kept)
        h2d(c, dst, src, n);
        return;
    }
    if (c->pend.empty()) c->pend_lo = c->stage_used;
    memcpy(c->h_stage + c->stage_used, src, n);
    c->pend.push_back(StageOp{(uint64_t)(uintptr_t)dst, (uint32_t)c->stage_used, (uint32_t)n, 0u, 0u});
    c->stage_used += (n + 63) & ~(size_t)63;
}
void stage_fill(mrg_ctx *c, void *dst, int byte, size_t n) {
    if (!n) return;
    if (!stage_room(c, 0) || n > MRG_STAGE_MAX) {
        flush_stage(c);
        HIPCHK(hipMemsetAsync(dst, byte, n, c->stream));
        return;
    }
    if (c->pend.empty()) c->pend_lo = c->stage_used;
    c->pend.push_back(StageOp{(uint64_t)(uintptr_t)dst, 0xFFFFFFFFu, (uint32_t)n, (uint32_t)(byte & 0xFF), 0u});
}

void read_counters(mrg_ctx *c) {
    HIPCHK(hipMemcpyAsync(c->h_cnt, c->d_cnt, sizeof(unsigned long long) * CNT_N, hipMemcpyDeviceToHost, c->stream));
    sync(c);
}

void ev_rec(mrg_ctx *c, int i) {
    if (c->timing) HIPCHK(hipEventRecord(c->ev[i], c->stream));
}
double ev_ms(mrg_ctx *c, int a, int b) {
    if (!c->timing) return 0.0;
    float ms = 0;
    HIPCHK(hipEventSynchronize(c->ev[b]));
    HIPCHK(hipEventElapsedTime(&ms, c->ev[a], c->ev[b]));
    return ms;
}

void keys_release(mrg_ctx *c) {
    KeysBuf &k = c->keys;
    Pool &p = c->pool;
    p.put(k.ks.k0); p.put(k.ks.k1); p.put(k.ks.cnt); p.put(k.ks.hoff);
    p.put(k.ks.doc); p.put(k.ks.len); p.put(k.ks.part);
    p.put(k.heap);
    k = KeysBuf{};
}

void keys_reserve(mrg_ctx *c, uint64_t cap) {
    keys_release(c);
    KeysBuf &k = c->keys;
    Pool &p = c->pool;
    k.ks.k0 = pget<uint64_t>(p, cap);
    k.ks.k1 = pget<uint64_t>(p, cap);
    k.ks.cnt = pget<uint64_t>(p, cap);
    k.ks.hoff = pget<uint64_t>(p, cap);
    k.ks.doc = pget<uint32_t>(p, cap);
    k.ks.len = pget<uint32_t>(p, cap);
    k.ks.part = pget<uint32_t>(p, cap);
    k.cap = cap;
}

uint64_t pow2_at_least(uint64_t x) {
    uint64_t p = 1024;
    while (p < x) p <<= 1;
    return p;
}

struct ShortSrc {
    const uint64_t *k0 = nullptr, *k1 = nullptr;
    const uint32_t *cnt = nullptr, *doc = nullptr;
    const XRec *x = nullptr;   // exchange records (short form only; long ones take the long path)
    const LRec *lx = nullptr;  // text-reduce line records
    uint64_t n = 0;
};

// Sum short-key records in the HBM table (exact; device-scope CAS) and append the distinct keys to
// c->keys (counter CNT_KEYS, which the caller has initialised).
void table_aggregate(mrg_ctx *c, const ShortSrc &src) {
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const bool idx = is_idx(c);
    if (src.n) {
        TableArgs T{};
        T.cap = pow2_at_least(2 * src.n);
        T.tk0 = pget<uint64_t>(p, T.cap);
        T.tk1 = pget<uint64_t>(p, T.cap);
        T.tcnt = pget<uint64_t>(p, T.cap);
        T.tdoc = idx ? pget<uint32_t>(p, T.cap) : nullptr;
        T.hash_bits = hash_bits(c);
        mrg_launch_table_clear(T, idx, s);
        if (src.x) mrg_launch_table_insert_x(T, src.x, src.n, idx, s);
        else if (src.lx) mrg_launch_table_insert_l(T, src.lx, src.n, idx, s);
        else mrg_launch_table_insert(T, src.k0, src.k1, src.cnt, src.doc, src.n, idx, s);
        mrg_launch_table_compact(T, idx, c->keys.ks, &c->d_cnt[CNT_KEYS], s);
        p.put(T.tk0); p.put(T.tk1); p.put(T.tcnt); p.put(T.tdoc);
    }
}

// Long keys: fingerprint sort + full-byte tie-break grouping; appends to c->keys and owns the heap.
void long_aggregate(mrg_ctx *c, LongItems li) {
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const bool idx = is_idx(c);
    if (li.n) {
        const uint64_t n = li.n;
        uint64_t *k0 = pget<uint64_t>(p, n), *k1 = pget<uint64_t>(p, n), *fp = pget<uint64_t>(p, n);
        uint64_t *fl64 = pget<uint64_t>(p, n), *hoff = pget<uint64_t>(p, n), *acc = pget<uint64_t>(p, n);
        uint32_t *fl = pget<uint32_t>(p, n), *ix = pget<uint32_t>(p, n), *rep = pget<uint32_t>(p, n);
        uint64_t *scantmp = pget<uint64_t>(p, mrg_scan_tmp_elems(n));
        mrg_launch_long_prep(li.base, li.start, li.rawlen, n, k0, k1, fl, fl64, fp, hash_bits(c), li.verbatim, s);
        mrg_scan_u64(fl64, hoff, n, scantmp, s);
        uint64_t last[2];
        HIPCHK(hipMemcpyAsync(&last[0], hoff + (n - 1), 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&last[1], fl64 + (n - 1), 8, hipMemcpyDeviceToHost, s));
        sync(c);
        const uint64_t heap_bytes = last[0] + last[1];
        c->keys.heap = pget<uint8_t>(p, heap_bytes + 16);
        c->keys.heap_bytes = heap_bytes;
        mrg_launch_long_gather(li.base, li.start, li.rawlen, n, hoff, c->keys.heap, li.verbatim, s);
        // fingerprint sort (collision-safe: k_long_group compares full bytes inside equal runs)
        uint64_t *fps = pget<uint64_t>(p, n);
        HIPCHK(hipMemcpyAsync(fps, fp, 8 * n, hipMemcpyDeviceToDevice, s));
        mrg_launch_iota_u32(ix, n, s);
        uint64_t *kv = pget<uint64_t>(p, 4 * n);
        void *stmp = p.get(mrg_sort_tmp_bytes(n));
        check_sort_n(n, "long-key fingerprint sort");
        mrg_radix_sort_u64(fps, ix, kv, n, stmp, s);
        mrg_launch_long_group(fps, ix, idx ? li.doc : nullptr, c->keys.heap, hoff, fl, n, rep, s);
        HIPCHK(hipMemsetAsync(acc, 0, 8 * n, s));
        mrg_launch_long_emit(rep, li.cnt, k0, k1, fl, hoff, li.doc, n, (unsigned long long *)acc, c->keys.ks,
                             &c->d_cnt[CNT_KEYS], idx, s);
        p.put(k0); p.put(k1); p.put(fp); p.put(fl64); p.put(hoff); p.put(acc);
        p.put(fl); p.put(ix); p.put(rep); p.put(scantmp); p.put(fps); p.put(kv); p.put(stmp);
        c->keys.any_long = true;
    }
}

// Distinct-key count + partition of every key (worker.rs:129).
// Keys [0, parted) already carry their partition (the bucket aggregation computes it as it writes them).
void finish_keys(mrg_ctx *c, bool counters_fresh = false, uint64_t parted = 0) {
    if (!counters_fresh) read_counters(c);
    c->keys.n = c->h_cnt[CNT_KEYS];
    if (c->keys.n > c->keys.cap) raise(MRG_EINVAL, "internal: key set overflow");
    if (parted < c->keys.n) {
        KeySet rest = c->keys.ks;  // SoA: the same arrays from key `parted` on (the heap offsets are absolute)
        rest.k0 += parted; rest.k1 += parted; rest.cnt += parted; rest.hoff += parted;
        rest.doc += parted; rest.len += parted; rest.part += parted;
        mrg_launch_partition(rest, c->keys.heap, c->keys.n - parted, c->R, c->stream);
    }
    c->st.distinct_keys = c->keys.n;
}

// Records that arrive as exchange records (shuffle import / plugin reduce): table + long path.
void aggregate(mrg_ctx *c, const ShortSrc &src, LongItems li) {
    keys_reserve(c, src.n + li.n + 1);
    HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_KEYS], 0, sizeof(unsigned long long), c->stream));
    table_aggregate(c, src);
    long_aggregate(c, li);
    finish_keys(c);
}

struct MapBufs {
    uint64_t *pool = nullptr, *rbase = nullptr;
    uint32_t *bcap = nullptr, *bcount = nullptr;
    uint64_t *pool16 = nullptr, *rbase16 = nullptr;
    uint32_t *bcap16 = nullptr, *bcount16 = nullptr;
    MapArgs *dargs = nullptr;
    uint64_t *ovf = nullptr;
    uint32_t *onext = nullptr;
    uint64_t *fk0 = nullptr, *fk1 = nullptr;
    uint32_t *fcnt = nullptr, *fdoc = nullptr, *foff = nullptr;
    uint64_t *lstart = nullptr;
    uint32_t *llen = nullptr, *ldoc = nullptr, *lcount = nullptr;
    uint64_t *dstart = nullptr;  // long-token records packed densely after the map
    uint32_t *dlen = nullptr, *ddoc = nullptr;
    uint32_t *gbits = nullptr;
    unsigned long long *prof = nullptr;
    unsigned long long *pool_ctr = nullptr;  // the load-balance pool's part counters
    void release(Pool &p) {
        p.put(prof);
        p.put(pool_ctr);
        p.put(lcount); p.put(dstart); p.put(dlen); p.put(ddoc);
        p.put(pool); p.put(rbase); p.put(bcap); p.put(bcount); p.put(dargs); p.put(ovf); p.put(onext);
        p.put(pool16); p.put(rbase16); p.put(bcap16); p.put(bcount16);
        p.put(fk0); p.put(fk1); p.put(fcnt); p.put(fdoc); p.put(foff);
        p.put(lstart); p.put(llen); p.put(ldoc); p.put(gbits);
        *this = MapBufs{};
    }
};

struct MapSteal;
void set_steal(mrg_ctx *c, MapArgs &A, MapBufs &M, const MapSteal &ms, uint64_t n_chunks);

struct AggLaunch {
    BucketArgs B{};
    uint64_t nlong = 0;  // long keys the launch reserved key slots for
    bool c32 = false, live = false;
};

uint64_t agg_ocap(mrg_ctx *c) {
    uint64_t ocap = std::max<uint64_t>(c->ovf_hint, 1u << 20);
    if (const uint64_t t = env_u64("MRG_TEST_AGG_OCAP", 0)) ocap = t;  // test knob: force the regrow path
    return ocap;
}

// one launch of the per-bucket aggregation over the map's output (its overflow list is returned to
// the pool by agg_put); zero: clear the two counters it adds to (the map launch zeroed them)
AggLaunch agg_launch(mrg_ctx *c, const MapArgs &A, uint32_t nreg, uint32_t regcap, uint64_t ocap, uint32_t nsub,
                     uint64_t nlong, bool c32, bool zero) {
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const bool idx = is_idx(c);
    // every workgroup (bucket, sub-range) may emit a full table of keys
    keys_reserve(c, (uint64_t)MRG_NBUCKET * std::max<uint32_t>(nsub, 1u) * MRG_BA_CAP + ocap + nlong + 1);
    AggLaunch L;
    BucketArgs &B = L.B;
    B.pool = A.pool; B.rbase = A.rbase; B.bcap = A.bcap; B.bcount = A.bcount;
    B.pool16 = A.pool16; B.rbase16 = A.rbase16; B.bcap16 = A.bcap16; B.bcount16 = A.bcount16;
    B.movf = A.ovf; B.monext = A.onext; B.mocap = A.ocap;
    B.fk0 = A.fk0; B.fk1 = A.fk1; B.fcnt = A.fcnt; B.fdoc = A.fdoc; B.foff = A.foff;
    B.nreg = nreg; B.regcap = regcap;
    B.ok0 = pget<uint64_t>(p, ocap); B.ok1 = pget<uint64_t>(p, ocap);
    B.ocnt = pget<uint32_t>(p, ocap); B.odoc = idx ? pget<uint32_t>(p, ocap) : nullptr;
    B.ocap = ocap;
    B.out = c->keys.ks;
    B.counters = c->d_cnt;
    B.hash_bits = hash_bits(c);
    B.ablate = getenv("MRG_AGG_ABLATE") ? (uint32_t)atoi(getenv("MRG_AGG_ABLATE")) : 0u;
    B.nsub = nsub;
    B.kcap = c->keys.cap;
    B.n_reduce = c->R;
    if (zero) {
        HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_KEYS], 0, 8, s));
        HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_OVF2], 0, 8, s));
    }
    mrg_launch_bucket_agg(B, idx, c32, s);
    L.nlong = nlong;
    L.c32 = c32;
    L.live = true;
    return L;
}

void agg_put(mrg_ctx *c, AggLaunch &L) {
    if (!L.live) return;
    Pool &p = c->pool;
    p.put(L.B.ok0); p.put(L.B.ok1); p.put(L.B.ocnt); p.put(L.B.odoc);
    L.live = false;
}

// Map-side records: per-bucket LDS aggregation of tail chunks + flushed map tables, exact overflow
// through the HBM table, then the long keys.
// Returns false (nothing aggregated) when far more keys miss the per-bucket tables than the overflow
// path handles well (millions of distinct keys without the tail share that selects the wide path up
// front): the caller then runs the wide aggregation on the same map output.
// pre: a launch the caller made right behind the map (before its counters reached the host), used
// when its parameters still hold -- the counters read after the map are then already its own.
bool bucket_aggregate(mrg_ctx *c, const MapArgs &A, uint32_t nreg, uint32_t regcap, LongItems li,
                      AggLaunch *pre = nullptr) {
    if (nreg > 2048) raise(MRG_EINVAL, "internal: %u map workgroups exceed the aggregation's region table", nreg);
    const bool idx = is_idx(c);
    uint64_t ocap = agg_ocap(c);
    uint32_t agg_launches = 0;
    uint32_t nsub = c->agg_nsub;
    if (const uint64_t t = env_u64("MRG_TEST_AGG_NSUB", 0)) nsub = (uint32_t)t;
    const bool dirty = pre && pre->live;  // a launch since the map: its counters need clearing before another
    for (;;) {
        ++agg_launches;
        // 32-bit LDS counts (larger table) when no key can reach 2^32: fewer tokens than that
        const bool c32 = c->h_cnt[CNT_TOKENS] < 0xFFFFFFFFull && nreg <= 512;
        AggLaunch L;
        // the queued launch is reused only when it ran with this job's parameters: sub-ranges, overflow
        // capacity, count width, and key slots for at least the long keys the map produced (the map
        // reruns whenever its long keys exceed their capacity, which drops the queued launch, so li.n <= nlong
        // holds here; it is checked rather than assumed)
        if (pre && pre->live && agg_launches == 1 && pre->B.nsub == nsub && pre->B.ocap == ocap &&
            li.n <= pre->nlong &&
            pre->B.kcap >= (uint64_t)MRG_NBUCKET * std::max<uint32_t>(nsub, 1u) * MRG_BA_CAP + ocap + li.n + 1 &&
            pre->c32 == c32) {
            L = *pre;  // its counters came with the map's
            pre->live = false;
            c->st.spec_agg = 1;
        } else {
            if (pre && pre->live) c->st.spec_agg = 2;
            if (pre) agg_put(c, *pre);
            L = agg_launch(c, A, nreg, regcap, ocap, nsub, li.n, c32, agg_launches > 1 || dirty);
            read_counters(c);
        }
        BucketArgs &B = L.B;
        if (c->h_cnt[CNT_KEYS] > c->keys.cap)
            raise(MRG_EINVAL, "internal: bucket aggregation emitted %llu keys for %llu slots",
                  (unsigned long long)c->h_cnt[CNT_KEYS], (unsigned long long)c->keys.cap);
        const uint64_t novf = c->h_cnt[CNT_OVF2];
        if (getenv("MRG_DEBUG"))
            fprintf(stderr, "[mrgpu] bucket agg: %llu keys, %llu overflow records (cap %llu)\n",
                    (unsigned long long)c->h_cnt[CNT_KEYS], (unsigned long long)novf, (unsigned long long)ocap);
        // Many keys missed the tables (more distinct keys per bucket than a table holds): split every
        // bucket over more workgroups (each reads the whole bucket and keeps one hash sub-range), up
        // to 16; the count is remembered by the context.  Beyond that, the wide aggregation.
        const uint64_t heavy = env_u64("MRG_TEST_AGG_WIDE_OVF", 4ull << 20);
        if (novf > heavy && nsub < 16 && !env_u64("MRG_TEST_AGG_NSUB", 0)) {
            agg_put(c, L);
            nsub = c->agg_nsub = std::min<uint32_t>(16, 2 * nsub);  // overflow counts records, not keys: double
            if (getenv("MRG_DEBUG")) fprintf(stderr, "[mrgpu] bucket agg: %llu overflow records -> %u workgroups per bucket\n", (unsigned long long)novf, nsub);
            continue;
        }
        const char *wenv = getenv("MRG_WIDE");  // MRG_WIDE=0 pins the bucket path (tests of its overflow)
        if (!idx && novf > heavy && !(wenv && atoi(wenv) == 0)) {
            agg_put(c, L);
            c->agg_nsub = 1;  // the next job starts from one workgroup per bucket (a low-cardinality job
                              // would otherwise stream every bucket 16 times)
            if (getenv("MRG_DEBUG")) fprintf(stderr, "[mrgpu] bucket agg: %llu overflow records -> wide\n", (unsigned long long)novf);
            return false;
        }
        if (novf > ocap) {  // overflow list too small: grow (remembered) and run again
            agg_put(c, L);
            ocap = c->ovf_hint = novf + novf / 8 + 1024;
            continue;
        }
        if (novf) {
            ShortSrc src;
            src.k0 = B.ok0; src.k1 = B.ok1; src.cnt = B.ocnt; src.doc = B.odoc; src.n = novf;
            table_aggregate(c, src);
        }
        agg_put(c, L);
        c->st.overflow_keys = novf;
        c->st.agg_launches = agg_launches;
        c->spec_agg = !idx;
        c->spec_c32 = c32;  // the width this job allowed (not the one a reused launch happened to use)
        c->st.agg_path = 1;
        c->wide_hint = false;
        {  // the next job's workgroups per bucket: enough sub-ranges for this job's key count, each
           // sub-range's table at most 5/6 full.  Each sub-range is one more pass over the bucket's
           // tail stream: zipf_u (2.9 M keys) aggregates in 6.9 ms at 1 (2 M records overflow to the
           // HBM table), 3.6 ms at 2 (81 % full, no overflow), 4.2 ms at 3 (profiles/r04/v34_*)
            const uint64_t slots = idx ? 4096u : (c32 ? 6912u : 6112u);  // k_keys.hip ba_cap
            const uint64_t per = (uint64_t)MRG_NBUCKET * (slots * 5u / 6u);
            c->agg_nsub = (uint32_t)std::min<uint64_t>(16, std::max<uint64_t>(1, (c->h_cnt[CNT_KEYS] + per - 1) / per));
        }
        break;
    }
    // the counters read after the aggregation are still current unless more keys were appended; the
    // keys it wrote already carry their partition
    const bool fresh = c->st.overflow_keys == 0 && li.n == 0;
    const uint64_t parted = std::min<uint64_t>(c->h_cnt[CNT_KEYS], c->keys.cap);
    long_aggregate(c, li);
    finish_keys(c, fresh, parted);
    return true;
}

uint32_t bytes_for(uint64_t maxval) {
    uint32_t b = 0;
    while (maxval) { ++b; maxval >>= 8; }
    return b;
}

// Wide (sort-based) aggregation for high-cardinality inputs (k_keys.hip k_wide_*): every map
// record is gathered with its partition, sorted by (partition, key) and summed per key; the key set
// comes out in output order.
void wide_aggregate_radix(mrg_ctx *c, const MapArgs &A, uint32_t nreg, uint32_t regcap, LongItems li) {
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    BucketArgs B{};
    B.pool = A.pool; B.rbase = A.rbase; B.bcap = A.bcap; B.bcount = A.bcount;
    B.pool16 = A.pool16; B.rbase16 = A.rbase16; B.bcap16 = A.bcap16; B.bcount16 = A.bcount16;
    B.movf = A.ovf; B.monext = A.onext; B.mocap = A.ocap;
    B.fk0 = A.fk0; B.fk1 = A.fk1; B.fcnt = A.fcnt; B.fdoc = A.fdoc; B.foff = A.foff;
    B.nreg = nreg; B.regcap = regcap;
    const uint64_t nseg = 2ull * nreg * MRG_NBUCKET + nreg + MRG_NBUCKET;
    uint64_t *segc = pget<uint64_t>(p, nseg + 1), *sego = pget<uint64_t>(p, nseg + 1);
    uint64_t *stmp1 = pget<uint64_t>(p, mrg_scan_tmp_elems(nseg + 1));
    HIPCHK(hipMemsetAsync(segc + nseg, 0, 8, s));
    mrg_launch_wide_counts(B, segc, nseg, s);
    mrg_scan_u64(segc, sego, nseg + 1, stmp1, s);  // sego[nseg] = total
    uint64_t n = 0;
    HIPCHK(hipMemcpyAsync(&n, sego + nseg, 8, hipMemcpyDeviceToHost, s));
    sync(c);
    SortRec *a = pget<SortRec>(p, std::max<uint64_t>(n, 1)), *b = pget<SortRec>(p, std::max<uint64_t>(n, 1));
    mrg_launch_wide_gather(B, sego, nseg, c->R, a, s);
    p.put(segc); p.put(sego); p.put(stmp1);
    SortPlan plan{};
    plan.use_part = c->R > 1;
    plan.part_bytes = bytes_for(c->R - 1);
    plan.use_k0 = plan.use_k1 = true;
    void *stmp = p.get(mrg_sort_tmp_bytes(n));
    int passes = 0;
    check_sort_n(n, "wide aggregation");
    SortRec *r = mrg_radix_sort(a, b, n, plan, stmp, s, &passes);
    p.put(stmp);
    uint64_t *head = pget<uint64_t>(p, n + 1), *cv = pget<uint64_t>(p, n + 1);
    uint64_t *E = pget<uint64_t>(p, n + 1), *C = pget<uint64_t>(p, n + 1);
    uint64_t *stmp2 = pget<uint64_t>(p, mrg_scan_tmp_elems(n + 1));
    mrg_launch_wide_heads(r, n, head, cv, s);
    mrg_scan_u64(head, E, n, stmp2, s);
    mrg_scan_u64(cv, C, n, stmp2, s);
    uint64_t tail[4] = {0, 0, 0, 0};
    if (n) {
        HIPCHK(hipMemcpyAsync(&tail[0], E + (n - 1), 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&tail[1], head + (n - 1), 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&tail[2], C + (n - 1), 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&tail[3], cv + (n - 1), 8, hipMemcpyDeviceToHost, s));
    }
    sync(c);
    const uint64_t runs = tail[0] + tail[1], ctot = tail[2] + tail[3];
    keys_reserve(c, runs + li.n + 1);
    uint64_t *F = pget<uint64_t>(p, runs + 1);
    mrg_launch_wide_keys(r, n, head, E, c->keys.ks, F, s);
    mrg_launch_wide_cnt(F, runs, n, C, ctot, c->keys.ks, s);
    HIPCHK(hipMemcpyAsync(&c->d_cnt[CNT_KEYS], &runs, 8, hipMemcpyHostToDevice, s));
    sync(c);  // `runs` is a host local
    p.put(a); p.put(b); p.put(head); p.put(cv); p.put(E); p.put(C); p.put(stmp2); p.put(F);
    c->st.overflow_keys = 0;
    c->keys.sorted = li.n == 0;
    long_aggregate(c, li);
    finish_keys(c);
}

// The wide result as a dense KeySet (sorted by partition and key) for the consumers other than the
// line writer (export, final.txt, long keys appended); `extra` more slots are reserved.
void wide_densify(mrg_ctx *c, uint64_t extra) {
    WideRes &w = c->wide;
    if (!w.ready) return;
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint64_t nl = (uint64_t)w.B1 * MRG_WIDE_MAXB2;
    uint32_t *doff = pget<uint32_t>(p, nl + 1);
    uint32_t *tmp = pget<uint32_t>(p, mrg_scan_tmp_elems(nl + 1));
    mrg_scan_u32(w.leaf_nd, doff, nl, tmp, s);
    keys_reserve(c, w.distinct + extra + 1);
    mrg_wide_launch_dense(w.kout, w.ocnt, w.leaf_pk, w.leaf_out, w.leaf_nd, doff, w.B1, w.B1r, c->keys.ks, s);
    HIPCHK(hipMemcpyAsync(&c->d_cnt[CNT_KEYS], &w.distinct, 8, hipMemcpyHostToDevice, s));
    sync(c);
    p.put(doff);
    p.put(tmp);
    c->keys.n = w.distinct;
    c->keys.sorted = true;
    w.release(p);
}

// Wide aggregation by the two-level sample sort (k_wide.hip): the map's count-1 records go through
// L1 (partition + global quantile splitters) and L2 (per-bucket splitters) into leaves; the flushed
// map-table entries (weighted) are aggregated apart, sorted, and merged into their leaves.
// The wide aggregation after L1: L2 leaves inside every L1 bucket (input: the L1 output K1 in bucket
// order with bstart, or -- rin != null -- the wide map's regions, segments soff), the leaves, the
// overflowing leaves' fallback, then the long keys.  K1 becomes the output key array; bid holds the
// L2 leaf id of every record.  Takes ownership of K1 (kept in c->wide), bstart, spl1, bid, wk*.
void wide_finish(mrg_ctx *c, LongItems li, uint64_t n, uint64_t nw, uint32_t B1, uint32_t B1r, uint64_t *K1,
                 uint64_t *bstart, uint64_t *spl1, uint16_t *bid, uint64_t *wk0, uint64_t *wk1, uint64_t *wcnt,
                 uint32_t *wpart, bool dbg, hipEvent_t *pe, int &npe, const WmapIn &wm) {
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint32_t R = c->R;
    auto mark = [&]() {
        if (!dbg || npe >= 8) return;
        HIPCHK(hipEventCreate(&pe[npe]));
        HIPCHK(hipEventRecord(pe[npe++], s));
    };
    // ---- L2: leaves inside every L1 bucket
    const uint64_t NL = (uint64_t)B1 * MRG_WIDE_MAXB2;
    // the wide map's buckets: with MRG_WIDE_L2_SAMPLED=1, sparse leaves in K2 from a sampled histogram
    // (-1 % of C5's step for 1.6x its device memory, so not the default);
    // MRG_TEST_L2_CAP=<mul>,<add> sets the leaf capacities (small ones force the exact redo),
    // MRG_TEST_L2_MIN the smallest bucket that samples
    L2Sparse sp;
    sp.on = wm.rin != nullptr && env_u64("MRG_WIDE_L2_SAMPLED", 0) != 0;
    if (const char *e = getenv("MRG_TEST_L2_CAP")) {
        unsigned a = 8, d = 64;
        if (sscanf(e, "%u,%u", &a, &d) >= 1) { sp.capmul = a; sp.capadd = d; }
    }
    sp.sample_min = (uint32_t)env_u64("MRG_TEST_L2_MIN", sp.sample_min);  // (tests: sample small buckets)
    if (sp.on) {
        sp.redo_flags = pget<uint32_t>(p, B1);
        HIPCHK(hipMemsetAsync(sp.redo_flags, 0, 4ull * B1, s));
    }
    const uint64_t nrec2 = sp.on ? 9 * n / 4 + 16 : n + 1;  // K2 records
    uint64_t *K2 = pget<uint64_t>(p, 2 * nrec2 + 2);
    uint32_t *nleaf = pget<uint32_t>(p, B1);
    uint64_t *leaf_lo = pget<uint64_t>(p, NL + 1), *leaf_lb = pget<uint64_t>(p, 2 * NL + 2);
    uint64_t *leaf_hi = pget<uint64_t>(p, NL + 1), *leaf_dlo = pget<uint64_t>(p, NL + 1);
    // records per leaf: the wide map's digit leaves come out near the target (320: r05 v61; 256 when cut
    // from the sampled histogram, whose leaves vary more: r06 v09, v11), the sampled splitters' leaves
    // vary like 8-sample gaps (256 keeps most under the one-wave capacity)
    const uint32_t target = (uint32_t)env_u64("MRG_TEST_LEAF_TARGET", wm.rin ? (sp.on ? 256 : 320) : 256);
    mrg_wide_launch_l2(wm.rin ? nullptr : K1, K2, bstart, spl1, B1, B1r, target, nleaf, leaf_lo, leaf_hi, leaf_dlo, leaf_lb,
                       bid, s, wm, sp);
    p.put(sp.redo_flags);
    p.put(bid);
    mark();  // 4: L2
    // ---- leaves: aggregate + sort + line bytes (K1 becomes the output key array)
    WideRes &w = c->wide;
    w.release(p);
    w.B1 = B1;
    w.B1r = B1r;
    w.kout = K1;
    w.ocnt = pget<uint64_t>(p, n + nw + 1);
    w.nleaf = nleaf;
    w.leaf_out = pget<uint64_t>(p, NL);
    w.leaf_nd = pget<uint32_t>(p, NL + 1);
    w.leaf_bytes = pget<uint64_t>(p, NL + 1);
    w.leaf_last = pget<uint32_t>(p, NL);
    w.leaf_pk = pget<uint32_t>(p, NL);
    HIPCHK(hipMemsetAsync(w.leaf_pk, 0, 4 * NL, s));
    HIPCHK(hipMemsetAsync(w.leaf_nd, 0, 4 * (NL + 1), s));
    HIPCHK(hipMemsetAsync(w.leaf_bytes, 0, 8 * (NL + 1), s));
    uint32_t *ovf_list = pget<uint32_t>(p, NL);
    HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_KEYS], 0, 8, s));
    HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_OVF2], 0, 8, s));
    WideLeafArgs L{};
    L.kin = K2; L.kout = K1; L.bstart = bstart; L.nleaf = nleaf; L.leaf_lo = leaf_lo; L.leaf_lb = leaf_lb;
    L.leaf_hi = leaf_hi; L.leaf_dlo = leaf_dlo;
    L.B1r = B1r; L.R = R; L.wk0 = wk0; L.wk1 = wk1; L.wcnt = wcnt; L.wpart = wpart; L.nw = nw;
    L.maxd = (uint32_t)env_u64("MRG_TEST_LEAF_CAP", 0);
    L.ocnt = w.ocnt; L.leaf_out = w.leaf_out; L.leaf_nd = w.leaf_nd; L.leaf_bytes = w.leaf_bytes;
    L.leaf_last = w.leaf_last; L.ovf_list = ovf_list; L.ovf_n = &c->d_cnt[CNT_OVF2]; L.nkeys = &c->d_cnt[CNT_KEYS];
    L.wr = pget<uint64_t>(p, 2 * NL);
    L.prof = pget<unsigned long long>(p, 16);
    HIPCHK(hipMemsetAsync(L.prof, 0, 128, s));
    L.big_list = pget<uint32_t>(p, NL);
    L.big_n = pget<unsigned long long>(p, 1);
    L.leaf_pk = w.leaf_pk;
    // counts packed into the key slots of leaves whose keys are <= 12 bytes: every count fits 32 bits
    // when the job has fewer than 2^32 tokens (MRG_TEST_NO_PACK: the unpacked layout everywhere)
    L.pack = (c->h_cnt[CNT_TOKENS] < 0xFFFFFFFFull && !getenv("MRG_TEST_NO_PACK")) ? 1u : 0u;
    HIPCHK(hipMemsetAsync(L.big_n, 0, 8, s));
    mrg_wide_launch_leaf(L, B1, s);
    mark();  // 5: leaves
    read_counters(c);
    const uint64_t novf = c->h_cnt[CNT_OVF2];
    if (novf) mrg_wide_launch_fallback(L, ovf_list, (uint32_t)novf, p, s);
    mark();  // 6: fallback
    read_counters(c);
    w.distinct = c->h_cnt[CNT_KEYS];
    w.ready = true;
    if (dbg) {
        static const char *nm[] = {"weights", "splitters", "L1", "L2", "leaves", "fallback"};
        fprintf(stderr, "[mrgpu] wide phases (ms):");
        for (int i = 1; i < npe; ++i) {
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, pe[i - 1], pe[i]));
            fprintf(stderr, " %s %.2f", nm[i - 1], ms);
        }
        fprintf(stderr, "\n");
        for (int i = 0; i < npe; ++i) (void)hipEventDestroy(pe[i]);
        unsigned long long pr[16], nbig = 0;
        HIPCHK(hipMemcpy(pr, L.prof, sizeof pr, hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(&nbig, L.big_n, 8, hipMemcpyDeviceToHost));
        fprintf(stderr, "[mrgpu] wide: %llu passed to the workgroup kernel (%llu by size, %llu by bucket)\n", nbig,
                pr[6], pr[7]);
        {  // leaf sizes (records)
            std::vector<uint32_t> hn(B1);
            std::vector<uint64_t> hlo(NL), hhi(NL);
            HIPCHK(hipMemcpy(hn.data(), nleaf, 4ull * B1, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(hlo.data(), leaf_lo, 8ull * NL, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(hhi.data(), leaf_hi, 8ull * NL, hipMemcpyDeviceToHost));
            std::vector<uint64_t> sz;
            for (uint32_t bb = 0; bb < B1; ++bb)
                for (uint32_t j = 0; j < hn[bb]; ++j) {
                    const uint64_t lid = (uint64_t)bb * MRG_WIDE_MAXB2 + j;
                    sz.push_back(hhi[lid] - hlo[lid]);
                }
            std::sort(sz.begin(), sz.end());
            if (!sz.empty())
                fprintf(stderr, "[mrgpu] wide: %zu leaves, records p10 %llu p50 %llu p63 %llu p87 %llu p99 %llu max %llu\n",
                        sz.size(), (unsigned long long)sz[sz.size() / 10], (unsigned long long)sz[sz.size() / 2],
                        (unsigned long long)sz[sz.size() * 63 / 100], (unsigned long long)sz[sz.size() * 87 / 100],
                        (unsigned long long)sz[sz.size() * 99 / 100], (unsigned long long)sz.back());
        }
        if (pr[0] | pr[1] | pr[5])
            fprintf(stderr, "[mrgpu] leaf phase clocks (wave 0, all WGs): clear %.3g insert %.3g list %.3g digits %.3g "
                            "order %.3g write %.3g\n", (double)pr[0], (double)pr[1], (double)pr[2], (double)pr[3],
                    (double)pr[4], (double)pr[5]);
        if (pr[8] | pr[12])
            fprintf(stderr, "[mrgpu] one-wave leaf phase clocks (all waves): load %.3g bits %.3g digits %.3g order %.3g "
                            "runs %.3g stats %.3g\n", (double)pr[8], (double)pr[9], (double)pr[10], (double)pr[11],
                    (double)pr[12], (double)pr[13]);
        {
            unsigned long long l2[8];
            mrg_wide_l2_prof(l2);
            if (l2[6])
                fprintf(stderr, "[mrgpu] L2 phase clocks (thread 0, all WGs, cumulative): segs %.3g sample %.3g sort %.3g "
                                "index %.3g hist %.3g scan %.3g scatter %.3g\n", (double)l2[0], (double)l2[1],
                        (double)l2[2], (double)l2[3], (double)l2[4], (double)l2[5], (double)l2[6]);
        }
        if (pr[14])
            fprintf(stderr, "[mrgpu] one-wave leaves: digits used %.3g, largest digit bucket %.3g (sums)\n", (double)pr[14],
                    (double)pr[15]);
    }
    if (getenv("MRG_DEBUG"))
        fprintf(stderr, "[mrgpu] wide: %llu records, %llu weighted, B1 %u (x%u), %llu distinct, %llu leaves overflowed\n",
                (unsigned long long)n, (unsigned long long)nw, B1, B1r, (unsigned long long)w.distinct,
                (unsigned long long)novf);
    p.put(K2); p.put(leaf_lo); p.put(leaf_lb); p.put(leaf_hi); p.put(leaf_dlo); p.put(ovf_list); p.put(spl1); p.put(bstart);
    p.put(L.wr);
    p.put(L.prof); p.put(L.big_list); p.put(L.big_n);
    p.put(wk0); p.put(wk1); p.put(wcnt); p.put(wpart);
    c->st.overflow_keys = novf;
    c->keys.n = 0;
    c->st.distinct_keys = w.distinct;
    if (li.n) {  // long keys: the dense key set plus the long keys, sorted by the generic path
        wide_densify(c, li.n);
        long_aggregate(c, li);
        finish_keys(c);
        c->keys.sorted = false;
    }
}

void wide_aggregate(mrg_ctx *c, const MapArgs &A, uint32_t nreg, uint32_t regcap, LongItems li) {
    const uint32_t R = c->R;
    if (R > 4096 || getenv("MRG_WIDE_RADIX")) {  // the L1 histogram holds R x B1r buckets in LDS
        wide_aggregate_radix(c, A, nreg, regcap, li);
        return;
    }
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    BucketArgs B{};
    B.pool = A.pool; B.rbase = A.rbase; B.bcap = A.bcap; B.bcount = A.bcount;
    B.pool16 = A.pool16; B.rbase16 = A.rbase16; B.bcap16 = A.bcap16; B.bcount16 = A.bcount16;
    B.movf = A.ovf; B.monext = A.onext; B.mocap = A.ocap;
    B.fk0 = A.fk0; B.fk1 = A.fk1; B.fcnt = A.fcnt; B.fdoc = A.fdoc; B.foff = A.foff;
    B.nreg = nreg; B.regcap = regcap;
    // MRG_DEBUG: HIP-event time of each phase
    const bool dbg = getenv("MRG_DEBUG") != nullptr;
    hipEvent_t pe[8] = {};
    int npe = 0;
    auto mark = [&]() {
        if (!dbg || npe >= 8) return;
        HIPCHK(hipEventCreate(&pe[npe]));
        HIPCHK(hipEventRecord(pe[npe++], s));
    };
    mark();
    // ---- segment sizes: main (count 1) and flushed tables (weighted)
    const uint64_t nsm = 2ull * nreg * MRG_NBUCKET + MRG_NBUCKET;  // 12-byte regions, overflow lists, 16-byte regions
    uint64_t *cm = pget<uint64_t>(p, nsm + 1), *om = pget<uint64_t>(p, nsm + 1), *segptr = pget<uint64_t>(p, nsm);
    uint64_t *cf = pget<uint64_t>(p, nreg + 1), *of = pget<uint64_t>(p, nreg + 1);
    uint64_t *st1 = pget<uint64_t>(p, mrg_scan_tmp_elems(nsm + 1));
    HIPCHK(hipMemsetAsync(cm + nsm, 0, 8, s));
    HIPCHK(hipMemsetAsync(cf + nreg, 0, 8, s));
    mrg_wide_launch_counts(B, cm, segptr, cf, s);
    mrg_scan_u64(cm, om, nsm + 1, st1, s);
    mrg_scan_u64(cf, of, nreg + 1, st1, s);
    uint64_t nn[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(&nn[0], om + nsm, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&nn[1], of + nreg, 8, hipMemcpyDeviceToHost, s));
    sync(c);
    const uint64_t n = nn[0], nf = nn[1];
    if (n >= 0xFFFFFFF0ull) raise(MRG_ENOMEM, "wide aggregation: %llu records exceed one GPU's 32-bit record index",
                                  (unsigned long long)n);
    // ---- weighted keys: HBM-table aggregation of the flushed entries, sorted by (partition, key)
    uint64_t nw = 0;
    uint64_t *wk0 = pget<uint64_t>(p, nf + 1), *wk1 = pget<uint64_t>(p, nf + 1), *wcnt = pget<uint64_t>(p, nf + 1);
    uint32_t *wpart = pget<uint32_t>(p, nf + 1);
    if (nf) {
        uint64_t *fk0 = pget<uint64_t>(p, nf), *fk1 = pget<uint64_t>(p, nf);
        uint32_t *fc = pget<uint32_t>(p, nf);
        mrg_wide_launch_flush_gather(B, of, fk0, fk1, fc, s);
        KeySet ks{};
        ks.k0 = pget<uint64_t>(p, nf); ks.k1 = pget<uint64_t>(p, nf); ks.cnt = pget<uint64_t>(p, nf);
        ks.hoff = pget<uint64_t>(p, nf); ks.doc = pget<uint32_t>(p, nf); ks.len = pget<uint32_t>(p, nf);
        ks.part = pget<uint32_t>(p, nf);
        TableArgs T{};
        T.cap = pow2_at_least(2 * nf);
        T.tk0 = pget<uint64_t>(p, T.cap); T.tk1 = pget<uint64_t>(p, T.cap); T.tcnt = pget<uint64_t>(p, T.cap);
        T.hash_bits = hash_bits(c);
        HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_KEYS], 0, 8, s));
        mrg_launch_table_clear(T, false, s);
        mrg_launch_table_insert(T, fk0, fk1, fc, nullptr, nf, false, s);
        mrg_launch_table_compact(T, false, ks, &c->d_cnt[CNT_KEYS], s);
        read_counters(c);
        nw = c->h_cnt[CNT_KEYS];
        mrg_launch_partition(ks, nullptr, nw, R, s);
        SortRec *ra = pget<SortRec>(p, nw), *rb = pget<SortRec>(p, nw);
        void *stmp = p.get(mrg_sort_tmp_bytes(nw));
        mrg_launch_make_sortrec(ks, nw, nullptr, ra, s);
        SortPlan plan{};
        plan.use_part = R > 1;
        plan.part_bytes = bytes_for(R - 1);
        plan.use_k0 = plan.use_k1 = true;
        int passes = 0;
        SortRec *srt = mrg_radix_sort(ra, rb, nw, plan, stmp, s, &passes);
        mrg_wide_launch_weights(srt, nw, ks, wk0, wk1, wcnt, wpart, s);
        sync(c);
        p.put(fk0); p.put(fk1); p.put(fc); p.put(ks.k0); p.put(ks.k1); p.put(ks.cnt); p.put(ks.hoff); p.put(ks.doc);
        p.put(ks.len); p.put(ks.part); p.put(T.tk0); p.put(T.tk1); p.put(T.tcnt); p.put(ra); p.put(rb); p.put(stmp);
    }
    mark();  // 1: weighted keys done
    // ---- L1 buckets: R partitions x B1r quantile ranges of about 2^18 records
    uint32_t B1r = (uint32_t)std::min<uint64_t>((n + ((uint64_t)R << 18) - 1) / ((uint64_t)R << 18), 64);
    B1r = std::max<uint32_t>(1, std::min<uint32_t>(B1r, std::max<uint32_t>(1, 4096 / R)));
    const uint32_t B1 = R * B1r;
    uint64_t *spl1 = pget<uint64_t>(p, 2ull * R * B1r + 2);
    if (B1r > 1 && n) {
        const uint32_t S1 = (uint32_t)std::min<uint64_t>(64ull * B1, n);
        SortRec *sa = pget<SortRec>(p, S1), *sb = pget<SortRec>(p, S1);
        void *stmp = p.get(mrg_sort_tmp_bytes(S1));
        mrg_wide_launch_sample1(B, om, nsm, n, S1, R, sa, s);
        SortPlan plan{};
        plan.use_part = R > 1;
        plan.part_bytes = bytes_for(R - 1);
        plan.use_k0 = plan.use_k1 = true;
        int passes = 0;
        SortRec *srt = mrg_radix_sort(sa, sb, S1, plan, stmp, s, &passes);
        mrg_wide_launch_split1(srt, S1, R, B1r, spl1, s);
        sync(c);
        p.put(sa); p.put(sb); p.put(stmp);
    }
    mark();  // 2: splitters
    const uint32_t ntiles = (uint32_t)std::max<uint64_t>(1, (n + MRG_WIDE_T1 - 1) / MRG_WIDE_T1);
    uint32_t *cnt1 = pget<uint32_t>(p, (uint64_t)B1 * ntiles + 1);
    uint32_t *st2 = pget<uint32_t>(p, mrg_scan_tmp_elems((uint64_t)B1 * ntiles + 1));
    uint64_t *K1 = pget<uint64_t>(p, 2 * (n + nw) + 2);
    uint64_t *bstart = pget<uint64_t>(p, B1 + 1);
    uint16_t *bid = pget<uint16_t>(p, std::max<uint64_t>(n, 1));   // L1 bucket, then L2 leaf, of each record
    uint8_t *ix1 = getenv("MRG_TEST_NO_L1IX") ? nullptr : pget<uint8_t>(p, 260ull * R);
    if (n) {
        mrg_wide_launch_l1(B, om, segptr, nsm, n, spl1, R, B1r, cnt1, ntiles, K1, bid, ix1, false, s);
        mrg_scan_u32(cnt1, cnt1, (uint64_t)B1 * ntiles, st2, s);
        mrg_wide_launch_l1(B, om, segptr, nsm, n, spl1, R, B1r, cnt1, ntiles, K1, bid, nullptr, true, s);
    } else {
        HIPCHK(hipMemsetAsync(cnt1, 0, 4ull * B1 * ntiles, s));
    }
    mrg_wide_launch_bstart(cnt1, B1, ntiles, n, bstart, s);
    p.put(cnt1); p.put(st2); p.put(cm); p.put(om); p.put(cf); p.put(of); p.put(st1); p.put(segptr);
    if (ix1) p.put(ix1);
    mark();  // 3: L1
    wide_finish(c, li, n, nw, B1, B1r, K1, bstart, spl1, bid, wk0, wk1, wcnt, wpart, dbg, pe, npe, WmapIn{});
}

void need_job(mrg_ctx *c) {
    if (!c) raise(MRG_EINVAL, "null context");
    if (!c->job) raise(MRG_EINVAL, "no job: call mrg_job_begin first");
}

void job_begin(mrg_ctx *c, int app, uint32_t R, uint32_t flags) {
    if (app != MRG_APP_WC && app != MRG_APP_INDEXER) raise(MRG_EINVAL, "unknown app %d", app);
    if (R == 0) raise(MRG_EINVAL, "n_reduce must be > 0");
    sync(c);
    flush_stage(c);     // (nothing is pending between jobs: every map launch flushes first)
    c->stage_used = 0;  // the previous job's staged copies are done
    c->pend_lo = 0;
    keys_release(c);
    c->wide.release(c->pool);
    c->job = true;
    c->app = app;
    c->R = R;
    c->flags = flags;
    c->d_in = nullptr;
    c->doc_off.clear();
    c->doc_ids.clear();
    c->mapped = c->reduced = false;
    c->n_owners = 0;
    c->out_bytes = 0;
    c->extra_first = 0;
    c->part_off.assign(R + 1, 0);
    c->final_bytes = 0;
    c->finalized = false;
    c->st = mrg_stats{};
}

// ---- the wide map (near-unique keys, wc): the splitters first, from a sample of the input text, then
// a map that writes every short key to its L1 bucket (R partitions x B1r key ranges) -- the L1 count
// and scatter passes over the map's records (wide_aggregate) disappear; L2 reads the regions.
struct WideMapPlan {
    bool on = false, forced = false, w12 = false;
    bool repeats = false;     // a cold context's sample found repeats: the bucket path is the likely one
    uint64_t n16 = 0, S = 0;  // sampled keys of 13..16 bytes, samples
    uint32_t B1 = 0, B1r = 0;
    uint64_t *spl1 = nullptr;
    uint8_t *ix1 = nullptr;
};

// Sampled (k_wsample_text + k_wsample_dups, ~0.1 ms and one host wait) on every wc job of >= 64 MiB
// whose context has no measured path yet -- the first job of a fresh context, so every mrg_run_job and
// every one-shot worker call -- and when the context's last such job went the wide way (or
// MRG_WIDE_MAP=1).  Taken when the sample is near-unique: fewer than 1 in 16 sampled tokens repeat a
// sampled neighbour in key order.  (Until r05 only the hint sampled: a cold near-unique job ran the
// LDS-combine map, overflowed its tail regions, reran it and took the L1 count + scatter passes.)
WideMapPlan wide_map_plan(mrg_ctx *c, const uint64_t *d_doc_off, uint32_t nd, uint64_t total, int grid) {
    WideMapPlan P;
    const char *env = getenv("MRG_WIDE_MAP");
    P.forced = env && atoi(env) != 0;
    if (is_idx(c) || (env && atoi(env) == 0) || total == 0 || wide_forced_off()) return P;
    if (!P.forced && (total < (64ull << 20) || (c->wc_sized && !c->wide_hint))) return P;
    const uint32_t R = c->R;
    if (R > MRG_WMAP_MAXB1 || grid > 512) return P;
    uint32_t B1r = std::min<uint32_t>(64, std::max<uint32_t>(1, MRG_WMAP_MAXB1 / R));
    if (const uint64_t t = env_u64("MRG_TEST_WMAP_B1R", 0)) B1r = (uint32_t)std::min<uint64_t>(B1r, t);
    const uint32_t B1 = R * B1r;
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint32_t S = (uint32_t)std::min<uint64_t>(64ull * B1, 1u << 20);
    flush_stage(c);  // the document tables, read by the sampling kernels
    if (!P.forced && !c->wide_hint) {  // no hint (a cold context): the one-launch test on 8192 samples first
        const uint32_t S0 = std::min<uint32_t>(S, 8192);
        SortRec *s0 = pget<SortRec>(p, S0);
        unsigned long long *d0 = pget<unsigned long long>(p, 2);
        mrg_wide_launch_sample_text(c->d_in, d_doc_off, nd, total, S0, R, s0, s);
        mrg_wide_launch_sample_uniq(s0, S0, d0, s);
        unsigned long long *h0 = &c->h_cnt[CNT_N];  // pinned scratch
        HIPCHK(hipMemcpyAsync(h0, d0, 16, hipMemcpyDeviceToHost, s));
        sync(c);
        const unsigned long long rep = h0[0];
        p.put(s0); p.put(d0);
        if (rep * 16 >= S0) {  // repeats: the LDS combine pays
            P.repeats = true;
            return P;
        }
    }
    SortRec *sa = pget<SortRec>(p, S), *sb = pget<SortRec>(p, S);
    void *stmp = p.get(mrg_sort_tmp_bytes(S));
    unsigned long long *dups = pget<unsigned long long>(p, 2);
    HIPCHK(hipMemsetAsync(dups, 0, 16, s));
    mrg_wide_launch_sample_text(c->d_in, d_doc_off, nd, total, S, R, sa, s);
    SortPlan plan{};
    plan.use_part = R > 1;
    plan.part_bytes = bytes_for(R - 1);
    plan.use_k0 = plan.use_k1 = true;
    int passes = 0;
    SortRec *srt = mrg_radix_sort(sa, sb, S, plan, stmp, s, &passes);
    mrg_wide_launch_sample_dups(srt, S, dups, s);
    uint64_t *spl1 = pget<uint64_t>(p, 2ull * R * B1r + 2);
    uint8_t *ix1 = nullptr;
    if (B1r > 1) {
        mrg_wide_launch_split1(srt, S, R, B1r, spl1, s);
        if (B1r >= 5 && R <= MRG_WMAP_IXR) {
            ix1 = pget<uint8_t>(p, (uint64_t)MRG_WIDE_IX1 * R);
            mrg_wide_launch_l1ix(spl1, R, B1r, ix1, s);
        }
    }
    unsigned long long dh[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(dh, dups, 16, hipMemcpyDeviceToHost, s));
    sync(c);
    const unsigned long long nd_h = dh[0];
    p.put(sa); p.put(sb); p.put(stmp); p.put(dups);
    if (!P.forced && nd_h * 16 >= S) {  // repeats: the LDS combine pays
        p.put(spl1);
        p.put(ix1);
        c->wide_hint = false;
        return P;
    }
    P.on = true;
    // 12-byte regions when keys of 13..16 bytes are rare (under 1 in 256 sampled tokens): those go to
    // per-bucket lists of 16-byte records (MRG_TEST_WMAP_W12=0/1 overrides)
    P.n16 = dh[1];
    P.S = S;
    P.w12 = !c->w12_off && dh[1] * 256 < S;
    if (const char *e = getenv("MRG_TEST_WMAP_W12")) P.w12 = atoi(e) != 0;
    P.B1 = B1;
    P.B1r = B1r;
    P.spl1 = spl1;
    P.ix1 = ix1;
    return P;
}

// Load balance of a map launch: the last 1/16 of the blocks form a pool that a
// workgroup's waves take from once its equal share of the rest is done, at most steal_max blocks per
// workgroup -- so a workgroup maps at most per_wg_blocks blocks, and its per-workgroup capacities (tail
// and long-token regions, wide-map regions, the non-ASCII tile list) are sized for that (wg_scale x an
// equal share).  MRG_MAP_STEAL=0, or a small input: equal shares of every block, as before r06.
struct MapSteal {
    uint64_t n_static = 0;     // blocks in equal shares
    uint32_t steal_max = 0;    // pool blocks one workgroup may take
    uint64_t per_wg_blocks = 0;
    double wg_scale = 1.0;
};
MapSteal map_steal(uint64_t n_chunks, int grid) {
    MapSteal m;
    const uint64_t g = (uint64_t)std::max(grid, 1);
    const uint64_t div = env_u64("MRG_MAP_STEAL", 16);  // the pool is 1/div of the blocks (0: no pool)
    const uint64_t pool = div ? n_chunks / div : 0;
    if (pool == 0 || pool < env_u64("MRG_TEST_STEAL_MIN", 64 * g)) {  // nothing worth balancing (tests: any pool)
        m.n_static = n_chunks;
        m.per_wg_blocks = (n_chunks + g - 1) / g + 1;
        return m;
    }
    m.n_static = n_chunks - pool;
    m.steal_max = (uint32_t)(2 * pool / g + 1024);
    m.per_wg_blocks = (m.n_static + g - 1) / g + 1 + m.steal_max;
    m.wg_scale = (double)m.per_wg_blocks / ((double)n_chunks / (double)g);
    return m;
}

// the steal plan into a launch's arguments, with its pool counters (zeroed on the stream)
void set_steal(mrg_ctx *c, MapArgs &A, MapBufs &M, const MapSteal &ms, uint64_t n_chunks) {
    if (n_chunks * MRG_MAP_NSUB >= 0xFFFFFFFFull) raise(MRG_ENOMEM, "input too large for one map launch");
    A.n_static = ms.n_static;
    A.steal_max = ms.steal_max;
    A.pool_ctr = nullptr;
    if (ms.n_static < n_chunks) {
        if (!M.pool_ctr) M.pool_ctr = pget<unsigned long long>(c->pool, 8 * 16);
        stage_fill(c, M.pool_ctr, 0, 8ull * 8 * 16);
        A.pool_ctr = M.pool_ctr;
    }
}

void job_map_wide(mrg_ctx *c, WideMapPlan &wp, uint64_t *d_doc_off, uint64_t *d_cb, uint32_t *d_ids, uint32_t nd,
                  uint64_t n_chunks, uint64_t total, int grid, const std::vector<uint32_t> &ids) {
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint32_t B1 = wp.B1;
    // records per (bucket, workgroup) region: the splitters make the buckets about equal; a token per
    // ~10 input bytes, +30 %, or the last run's demand
    const MapSteal ms = map_steal(n_chunks, grid);
    uint64_t wcap = std::max<uint64_t>(c->wcap_hint,
                                       (uint64_t)(1.3 * ms.wg_scale * (double)total / 10.0 / (double)grid / (double)B1) + 64);
    if (const uint64_t t = env_u64("MRG_TEST_WMAP_CAP", 0)) wcap = t;
    uint64_t lcap = std::max<uint64_t>(c->long_hint, total / 1024 + 1024);
    MapArgs A{};
    MapBufs M;
    uint64_t *wrec = nullptr, *wl16 = nullptr;
    uint32_t *wcnt = nullptr, *wl16n = nullptr;
    uint32_t launches = 0;
    bool w12 = wp.w12;
    // the 16-byte lists of 12-byte regions: four times the sampled share of such keys, at least 2 K each
    uint64_t wl16cap = std::max<uint64_t>(2048, (uint64_t)(4.0 * (double)total / 10.0 / (double)B1 *
                                                            (double)(wp.n16 + 1) / (double)std::max<uint64_t>(wp.S, 1)));
    if (const uint64_t t = env_u64("MRG_TEST_WMAP_L16", 0)) wl16cap = t;
    for (;;) {
        if (wcap > 0xFFFFFFF0ull) raise(MRG_ENOMEM, "input too large for one map launch");
        M.dargs = pget<MapArgs>(p, 1);
        uint64_t lper = std::max<uint64_t>(c->lper_hint, (uint64_t)(ms.wg_scale * (double)((lcap + grid - 1) / grid)) + 16);
        const uint64_t lovf = lcap / 4 + 1024;
        const uint64_t lslots = (uint64_t)grid * lper + lovf;
        M.lstart = pget<uint64_t>(p, lslots);
        M.llen = pget<uint32_t>(p, lslots);
        M.ldoc = pget<uint32_t>(p, lslots);
        M.lcount = pget<uint32_t>(p, (uint64_t)grid);
        A = MapArgs{};
        A.kwords = (uint32_t)(MRG_MAP_NSUB * ms.per_wg_blocks);
        M.gbits = pget<uint32_t>(p, (uint64_t)grid * A.kwords);
        set_steal(c, A, M, ms, n_chunks);
        const uint64_t nslots = (uint64_t)B1 * grid * wcap;
        wrec = pget<uint64_t>(p, w12 ? (12 * nslots + 16 + 7) / 8 : 2 * nslots + 2);
        wcnt = pget<uint32_t>(p, (uint64_t)B1 * grid);
        if (w12) {
            if (wl16cap > 0xFFFFFFF0ull) raise(MRG_ENOMEM, "input too large for one map launch");
            wl16 = pget<uint64_t>(p, 2ull * B1 * wl16cap + 2);
            wl16n = pget<uint32_t>(p, B1);
            HIPCHK(hipMemsetAsync(wl16n, 0, 4ull * B1, s));
        }
        A.in = c->d_in;
        A.doc_off = d_doc_off;
        A.chunk_base = d_cb;
        A.doc_id = d_ids;
        A.n_docs = nd;
        A.n_chunks = n_chunks;
        A.lstart = M.lstart; A.llen = M.llen; A.ldoc = M.ldoc; A.lper = (uint32_t)lper; A.lovf = lovf;
        A.lcount = M.lcount;
        A.gbits = M.gbits;
        A.counters = c->d_cnt;
        A.hash_bits = hash_bits(c);
        A.wrec = wrec; A.wcnt = wcnt; A.wspl = wp.spl1; A.wix = wp.ix1;
        A.wR = c->R; A.wB1r = wp.B1r; A.wcap = (uint32_t)wcap;
        A.w12 = w12 ? 1u : 0u; A.wl16cap = (uint32_t)wl16cap; A.wl16 = wl16; A.wl16n = wl16n;
        // the kernel's LDS cursors, splitters and index rows are sized by these bounds (k_map.hip)
        if (A.wB1r == 0 || (uint64_t)A.wR * A.wB1r > MRG_WMAP_MAXB1 || (A.wix && A.wR > MRG_WMAP_IXR))
            raise(MRG_EINVAL, "wide map plan exceeds the kernel's LDS bounds");
        HIPCHK(hipMemsetAsync(c->d_cnt, 0, sizeof(unsigned long long) * CNT_N, s));
        HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_ERRPOS], 0xFF, sizeof(unsigned long long), s));
        flush_stage(c);  // (set_steal's pool counters)
        ev_rec(c, 0);
        h2d(c, M.dargs, &A, sizeof(MapArgs));
        mrg_launch_map(nullptr, M.dargs, c->app, grid, c->lds_cap, s, true);
        ev_rec(c, 1);
        HIPCHK(hipGetLastError());
        ++launches;
        read_counters(c);
        const uint64_t nl = c->h_cnt[CNT_LONG];
        const bool long_full = c->h_cnt[CNT_LONGX] > A.lovf;
        const bool l16_full = c->h_cnt[CNT_W16] != 0;
        if (c->h_cnt[CNT_OVF] == 0 && !long_full && !l16_full) break;
        if (l16_full) {  // too many keys of 13..16 bytes for the lists: 16-byte regions from now on
            w12 = false;
            c->w12_off = true;
        }
        if (c->h_cnt[CNT_OVF]) {  // a region overflowed: every region sized to the largest demand
            std::vector<uint32_t> wc((uint64_t)B1 * grid);
            HIPCHK(hipMemcpyAsync(wc.data(), wcnt, 4ull * wc.size(), hipMemcpyDeviceToHost, s));
            sync(c);
            const uint64_t mx = *std::max_element(wc.begin(), wc.end());
            wcap = c->wcap_hint = std::max<uint64_t>(wcap, mx + mx / 4 + 64);
        }
        if (long_full) {
            std::vector<uint32_t> lc((uint64_t)grid);
            HIPCHK(hipMemcpyAsync(lc.data(), M.lcount, 4ull * grid, hipMemcpyDeviceToHost, s));
            sync(c);
            const uint64_t mx = *std::max_element(lc.begin(), lc.end());
            c->lper_hint = mx + mx / 4 + 64;
            lcap = c->long_hint = std::max<uint64_t>(lcap, nl + nl / 8 + 1024);
        }
        if (getenv("MRG_DEBUG"))
            fprintf(stderr, "[mrgpu] wide map rerun: region overflow %llu (cap now %llu), long %llu\n",
                    (unsigned long long)c->h_cnt[CNT_OVF], (unsigned long long)wcap, (unsigned long long)nl);
        M.release(p);
        p.put(wrec); p.put(wcnt); p.put(wl16); p.put(wl16n);
        wl16 = nullptr;
        wl16n = nullptr;
    }
    c->st.ms_map = ev_ms(c, 0, 1);
    c->st.map_launches = launches;
    c->st.input_bytes = total;
    c->st.tokens = c->h_cnt[CNT_TOKENS];
    c->st.long_tokens = c->h_cnt[CNT_LONG];
    c->st.map_records = c->h_cnt[CNT_REC];
    c->st.nonascii_tiles = c->h_cnt[CNT_NONASCII];
    c->st.tail_records_16 = 0;
    c->st.map_spill = 0;
    const uint64_t errpos = c->h_cnt[CNT_ERRPOS];
    auto release_all = [&]() {
        M.release(p);
        p.put(wrec); p.put(wcnt); p.put(wl16); p.put(wl16n);
        p.put(d_doc_off); p.put(d_cb); p.put(d_ids);
    };
    if (errpos != ~0ull) {
        release_all();
        p.put(wp.spl1); p.put(wp.ix1);
        uint32_t d = 0;
        while (d + 1 < nd && c->doc_off[d + 1] <= errpos) ++d;
        raise(MRG_EUTF8, "stream did not contain valid UTF-8: document %u (id %u), byte offset %llu", d, ids[d],
              (unsigned long long)(errpos - c->doc_off[d]));
    }
    ev_rec(c, 2);
    LongItems li{};
    li.base = c->d_in; li.cnt = nullptr;
    li.n = c->h_cnt[CNT_LONG];
    if (li.n) {
        M.dstart = pget<uint64_t>(p, li.n);
        M.dlen = pget<uint32_t>(p, li.n);
        M.ddoc = pget<uint32_t>(p, li.n);
        mrg_launch_long_compact(A, grid, M.dstart, M.dlen, M.ddoc, s);
    }
    li.start = M.dstart; li.rawlen = M.dlen; li.doc = M.ddoc;
    // ---- the regions as L1 buckets: per-bucket segment starts, bucket offsets, then L2 and the leaves
    uint32_t *soff = pget<uint32_t>(p, (uint64_t)B1 * (grid + 2));
    uint64_t *nbk = pget<uint64_t>(p, (uint64_t)B1 + 1);
    uint64_t *bstart = pget<uint64_t>(p, (uint64_t)B1 + 1);
    uint64_t *tmp = pget<uint64_t>(p, mrg_scan_tmp_elems((uint64_t)B1 + 1));
    HIPCHK(hipMemsetAsync(nbk + B1, 0, 8, s));
    mrg_wmap_launch_seg(wcnt, B1, (uint32_t)grid, (uint32_t)wcap, w12 ? wl16n : nullptr, (uint32_t)wl16cap, soff, nbk, s);
    mrg_scan_u64(nbk, bstart, (uint64_t)B1 + 1, tmp, s);  // bstart[B1] = records
    uint64_t n = 0;
    HIPCHK(hipMemcpyAsync(&n, bstart + B1, 8, hipMemcpyDeviceToHost, s));
    sync(c);
    if (n >= 0xFFFFFFF0ull) raise(MRG_ENOMEM, "wide aggregation: %llu records exceed one GPU's 32-bit record index",
                                  (unsigned long long)n);
    uint64_t *K1 = pget<uint64_t>(p, 2 * n + 2);  // the leaves' output keys
    uint16_t *bid = pget<uint16_t>(p, std::max<uint64_t>(n, 1));
    uint64_t *wk0 = pget<uint64_t>(p, 1), *wk1 = pget<uint64_t>(p, 1), *wk = pget<uint64_t>(p, 1);
    uint32_t *wpart = pget<uint32_t>(p, 1);
    const bool dbg = getenv("MRG_DEBUG") != nullptr;
    hipEvent_t pe[8] = {};
    int npe = 0;
    c->st.agg_path = 2;
    c->spec_agg = false;
    WmapIn wm;
    wm.rin = wrec; wm.soff = soff; wm.grid = (uint32_t)grid; wm.wcap = (uint32_t)wcap;
    wm.w12 = w12 ? 1u : 0u; wm.wl16cap = (uint32_t)wl16cap; wm.wl16 = wl16;
    wide_finish(c, li, n, 0, B1, wp.B1r, K1, bstart, wp.spl1, bid, wk0, wk1, wk, wpart, dbg, pe, npe, wm);
    p.put(soff); p.put(nbk); p.put(tmp); p.put(wp.ix1);
    c->st.map_kind = 1;
    ev_rec(c, 3);
    release_all();
    c->st.ms_aggregate = ev_ms(c, 2, 3);
    // the hint holds while the input stays near-unique
    c->wide_hint = 2 * c->st.distinct_keys > c->st.tokens;
    c->wc_sized = true;
    c->mapped = true;
}

void job_map(mrg_ctx *c) {
    need_job(c);
    if (c->doc_off.empty()) raise(MRG_EINVAL, "no input: call mrg_job_set_input first");
    c->wide.release(c->pool);  // a second map of the same job replaces the first one's keys
    c->mapped = c->reduced = false;
    c->st.spec_agg = c->st.agg_path = c->st.map_kind = 0;
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint32_t nd = (uint32_t)c->doc_off.size() - 1;
    const uint64_t total = c->doc_off[nd] - c->doc_off[0];
    std::vector<uint64_t> cb(nd + 1, 0);
    for (uint32_t d = 0; d < nd; ++d) cb[d + 1] = cb[d] + mrg_map_tiles(c->doc_off[d], c->doc_off[d + 1]);
    const uint64_t n_chunks = cb[nd];
    std::vector<uint32_t> ids = c->doc_ids;
    if (ids.empty()) for (uint32_t d = 0; d < nd; ++d) ids.push_back(d);

    uint64_t *d_doc_off = pget<uint64_t>(p, nd + 1), *d_cb = pget<uint64_t>(p, nd + 1);
    uint32_t *d_ids = pget<uint32_t>(p, nd);
    stage_h2d(c, d_doc_off, c->doc_off.data(), 8ull * (nd + 1));
    stage_h2d(c, d_cb, cb.data(), 8ull * (nd + 1));
    stage_h2d(c, d_ids, ids.data(), 4ull * nd);

    if (!c->map_grid) c->map_grid = mrg_map_max_grid(c->app, c->lds_cap, c->device);
    // (MRG_TEST_MAP_GRID: more workgroups than fit at once, run in waves: an A/B knob for load balance)
    const uint64_t grid_want = env_u64("MRG_TEST_MAP_GRID", (uint64_t)c->map_grid);
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>(grid_want, n_chunks));
    bool cold_repeats = false;  // a cold context whose sample found repeats: queue the aggregation too
    {  // near-unique input: the wide map (every key straight to its L1 bucket)
        WideMapPlan wp = wide_map_plan(c, d_doc_off, nd, total, grid);
        if (wp.on) {
            job_map_wide(c, wp, d_doc_off, d_cb, d_ids, nd, n_chunks, total, grid, ids);
            return;
        }
        cold_repeats = wp.repeats;
    }
    const uint32_t cap = (uint32_t)mrg_map_cap(c->app, c->lds_cap);
    const bool idx = is_idx(c);
    const uint32_t RW = idx ? 3u : 2u;
    uint64_t lcap = std::max<uint64_t>(c->long_hint, total / 1024 + 1024);
    // records per (bucket, workgroup) tail region: ~1 in 20 input bytes is a tail record (combine
    // misses), spread evenly over the buckets; grown per bucket to the measured demand on a rerun
    const MapSteal ms = map_steal(n_chunks, grid);
    const double per_wg = (double)std::max<uint64_t>(total, 1) / grid * ms.wg_scale;
    // wc keys of 13..16 bytes (rare in text) get regions of 16-byte records a sixteenth that size
    std::vector<uint64_t> bcap(MRG_NBUCKET), bcap16(MRG_NBUCKET, 0);
    for (int b = 0; b < MRG_NBUCKET; ++b) {
        double est = per_wg / 20.0 / MRG_NBUCKET;
        if (c->bcap_rate.size() == MRG_NBUCKET) est = std::max(est, c->bcap_rate[b] * per_wg);
        bcap[b] = (uint64_t)(est * 1.25) + 32;
        if (!idx) {
            double est16 = per_wg / 20.0 / MRG_NBUCKET / 16.0;
            if (c->bcap16_rate.size() == MRG_NBUCKET) est16 = std::max(est16, c->bcap16_rate[b] * per_wg);
            bcap16[b] = (uint64_t)(est16 * 1.25) + 16;
        }
    }
    // per-bucket overflow lists absorb the run-to-run variation of the regions' demand (the LDS
    // table's contents depend on wave timing: a frequent key that finds its set full in one
    // workgroup sends all its tokens to one region), so a launch is repeated only when one fills
    // up.  Sized at a quarter of the default region total per bucket (C3: 2 GiB, only touched as
    // far as used); at 1/16 about one step in ten reran the whole map.
    uint64_t ocap = std::max<uint64_t>(c->ocap_hint, std::max<uint64_t>(1024, total / 20 / MRG_NBUCKET / 4));
    if (const uint64_t t = env_u64("MRG_TEST_TAIL_CAP", 0)) {  // test knobs
        bcap.assign(MRG_NBUCKET, t);
        if (!idx) bcap16.assign(MRG_NBUCKET, t);
    }
    if (const uint64_t t = env_u64("MRG_TEST_OVF_CAP", 0)) ocap = t;
    MapArgs A{};
    MapBufs M;
    AggLaunch spec;  // the aggregation launched right behind the map (wc, the last job took the bucket path)
    uint32_t launches = 0;
    for (;;) {
        std::vector<uint64_t> rbase(MRG_NBUCKET, 0), rbase16(MRG_NBUCKET, 0);
        std::vector<uint32_t> bcap32(MRG_NBUCKET), bcap16_32(MRG_NBUCKET);
        uint64_t rtot = 0, rtot16 = 0;
        for (int b = 0; b < MRG_NBUCKET; ++b) {
            if (bcap[b] > 0xFFFFFFF0ull || bcap16[b] > 0xFFFFFFF0ull)
                raise(MRG_ENOMEM, "input too large for one map launch");
            bcap32[b] = (uint32_t)bcap[b];
            rbase[b] = rtot;
            rtot += (uint64_t)grid * bcap[b];
            bcap16_32[b] = (uint32_t)bcap16[b];
            rbase16[b] = rtot16;
            rtot16 += (uint64_t)grid * bcap16[b];
        }
        M.rbase = pget<uint64_t>(p, MRG_NBUCKET);
        M.bcap = pget<uint32_t>(p, MRG_NBUCKET);
        M.bcount = pget<uint32_t>(p, (uint64_t)grid * MRG_NBUCKET);
        M.rbase16 = pget<uint64_t>(p, MRG_NBUCKET);
        M.bcap16 = pget<uint32_t>(p, MRG_NBUCKET);
        M.bcount16 = pget<uint32_t>(p, (uint64_t)grid * MRG_NBUCKET);
        M.dargs = pget<MapArgs>(p, 1);
        if (ocap > 0xFFFFFFF0ull) raise(MRG_ENOMEM, "input too large for one map launch");
        M.ovf = pget<uint64_t>(p, (uint64_t)MRG_NBUCKET * ocap * RW);
        M.onext = pget<uint32_t>(p, MRG_NBUCKET);
        stage_fill(c, M.onext, 0, 4ull * MRG_NBUCKET);
        stage_h2d(c, M.rbase, rbase.data(), 8ull * MRG_NBUCKET);
        stage_h2d(c, M.bcap, bcap32.data(), 4ull * MRG_NBUCKET);
        stage_h2d(c, M.rbase16, rbase16.data(), 8ull * MRG_NBUCKET);
        stage_h2d(c, M.bcap16, bcap16_32.data(), 4ull * MRG_NBUCKET);
        A.in = c->d_in;
        A.doc_off = d_doc_off;
        A.chunk_base = d_cb;
        A.doc_id = d_ids;
        A.n_docs = nd;
        A.n_chunks = n_chunks;
        // 12-byte (wc) / 24-byte (indexer) records, + 16 bytes: readers may load a 12-byte record as 16
        M.pool = pget<uint64_t>(p, (rtot * MRG_TAIL_BYTES(idx) + 16 + 7) / 8);
        M.pool16 = pget<uint64_t>(p, 2 * rtot16 + 2);
        M.fk0 = pget<uint64_t>(p, (uint64_t)grid * cap);
        M.fk1 = pget<uint64_t>(p, (uint64_t)grid * cap);
        M.fcnt = pget<uint32_t>(p, (uint64_t)grid * cap);
        M.fdoc = idx ? pget<uint32_t>(p, (uint64_t)grid * cap) : nullptr;
        M.foff = pget<uint32_t>(p, (uint64_t)grid * (MRG_NBUCKET + 1));
        // long tokens: per-workgroup regions of lper records + a shared list of lovf
        uint64_t lper = std::max<uint64_t>(c->lper_hint, (uint64_t)(ms.wg_scale * (double)((lcap + grid - 1) / grid)) + 16);
        uint64_t lovf = lcap / 4 + 1024;
        if (launches == 0) {  // test knobs (first launch only: a rerun grows them from the measured demand)
            if (const uint64_t t = env_u64("MRG_TEST_LONG_PER", 0)) lper = t;
            if (const uint64_t t = env_u64("MRG_TEST_LONG_LIST", 0)) lovf = t;
        }
        if (lper > 0xFFFFFFF0ull) raise(MRG_ENOMEM, "input too large for one map launch");
        const uint64_t lslots = (uint64_t)grid * lper + lovf;
        M.lstart = pget<uint64_t>(p, lslots);
        M.llen = pget<uint32_t>(p, lslots);
        M.ldoc = pget<uint32_t>(p, lslots);
        M.lcount = pget<uint32_t>(p, (uint64_t)grid);
        A.pool = M.pool; A.rbase = M.rbase; A.bcap = M.bcap; A.bcount = M.bcount;
        A.pool16 = M.pool16; A.rbase16 = M.rbase16; A.bcap16 = M.bcap16; A.bcount16 = M.bcount16;
        A.ovf = M.ovf; A.onext = M.onext; A.ocap = (uint32_t)ocap;
        A.fk0 = M.fk0; A.fk1 = M.fk1; A.fcnt = M.fcnt; A.fdoc = M.fdoc; A.foff = M.foff;
        A.lstart = M.lstart; A.llen = M.llen; A.ldoc = M.ldoc; A.lper = (uint32_t)lper; A.lovf = lovf;
        A.lcount = M.lcount;
        {  // non-ASCII tile lists: one entry per tile of a workgroup's share and steal budget at most
            A.kwords = (uint32_t)(MRG_MAP_NSUB * ms.per_wg_blocks);
            M.gbits = pget<uint32_t>(p, (uint64_t)grid * A.kwords);
            A.gbits = M.gbits;
        }
        set_steal(c, A, M, ms, n_chunks);
        A.counters = c->d_cnt;
        A.hash_bits = hash_bits(c);
        A.ablate = getenv("MRG_ABLATE") ? (uint32_t)atoi(getenv("MRG_ABLATE")) : 0u;
        A.prof = nullptr;
        if (getenv("MRG_PROF")) {
            M.prof = pget<unsigned long long>(p, 8 + 8ull * grid);
            HIPCHK(hipMemsetAsync(M.prof, 0, 8ull * (8 + 8ull * grid), s));
            A.prof = M.prof;
        }
        stage_fill(c, c->d_cnt, 0, sizeof(unsigned long long) * CNT_N);
        stage_fill(c, &c->d_cnt[CNT_ERRPOS], 0xFF, sizeof(unsigned long long));
        stage_h2d(c, M.dargs, &A, sizeof(MapArgs));
        flush_stage(c);
        ev_rec(c, 0);
        mrg_launch_map(nullptr, M.dargs, c->app, grid, c->lds_cap, s);  // also with no tiles: writes empty flush regions
        ev_rec(c, 1);
        HIPCHK(hipGetLastError());
        ++launches;
        // the aggregation queued behind the map before the host sees the map's counters (one host
        // round trip less per job); checked against them below and by bucket_aggregate, and dropped
        // when the map reruns, goes wide or the 32-bit-count guess was wrong
        // (MRG_WIDE=1 forces the wide path, so nothing is queued; MRG_WIDE=0 and MRG_TEST_AGG_NSUB still
        // queue it: their tests run through this path)
        // (r06: also on a cold context's first job when its sample found repeats; the 32-bit-count guess
        // is then "fewer than 2^32 tokens" -- true unless the input holds billions of one-letter words --
        // and bucket_aggregate checks it like every guess: a wrong one only drops the queued launch)
        if (launches == 1 && !idx && (c->spec_agg || cold_repeats) && !M.prof && !wide_forced() &&
            !getenv("MRG_NO_SPEC_AGG") && grid <= 2048) {
            ev_rec(c, 2);
            uint32_t nsub = c->agg_nsub;
            if (const uint64_t t = env_u64("MRG_TEST_AGG_NSUB", 0)) nsub = (uint32_t)t;
            const bool c32 = c->spec_agg ? c->spec_c32 : true;
            spec = agg_launch(c, A, (uint32_t)grid, cap, agg_ocap(c), nsub, lslots, c32 && grid <= 512, false);
        }
        // overflow-list fill into pinned scratch, then the counters: one host wait for both
        uint32_t *onext = (uint32_t *)&c->h_cnt[CNT_N + 8];
        HIPCHK(hipMemcpyAsync(onext, M.onext, 4ull * MRG_NBUCKET, hipMemcpyDeviceToHost, s));
        read_counters(c);
        c->st.map_spill = 0;
        for (int b = 0; b < MRG_NBUCKET; ++b) c->st.map_spill += std::min<uint64_t>(onext[b], ocap);
        if (M.prof) {
            unsigned long long pr[8];
            HIPCHK(hipMemcpy(pr, M.prof, sizeof pr, hipMemcpyDeviceToHost));
            double tot = 0;
            for (int i = 0; i < 7; ++i) tot += (double)pr[i];
            static const char *nm[7] = {"load-wait", "classify", "stage+scan+queue", "token rounds", "slow tokens",
                                        "non-ascii", "flush"};
            fprintf(stderr, "[mrgpu] map phase clocks (sum over waves %.3e):", tot);
            for (int i = 0; i < 7; ++i) fprintf(stderr, " %s %.1f%%", nm[i], 100.0 * (double)pr[i] / (tot > 0 ? tot : 1));
            fprintf(stderr, "\n");
            // workgroup start/end wall clocks (100 MHz; written by -DMRG_MAP_PROF builds only)
            std::vector<unsigned long long> wt(8ull * grid);
            HIPCHK(hipMemcpy(wt.data(), M.prof + 8, 8ull * wt.size(), hipMemcpyDeviceToHost));
            if (wt[1]) {
                unsigned long long t0 = ~0ull, t1 = 0, ls = 0;
                std::vector<double> dur(grid), end(grid), lend(grid);
                std::vector<std::vector<double>> fst(5, std::vector<double>(grid, 0.0));
                for (int g = 0; g < grid; ++g) t0 = std::min(t0, wt[8 * g]);
                for (int g = 0; g < grid; ++g) {
                    const unsigned long long *w = &wt[8ull * g];
                    t1 = std::max(t1, w[1]);
                    ls = std::max(ls, w[0]);
                    dur[g] = (double)(w[1] - w[0]) * 1e-5;
                    end[g] = (double)(w[1] - t0) * 1e-5;
                    lend[g] = w[2] ? (double)(w[2] - t0) * 1e-5 : 0.0;
                    unsigned long long prev = w[2];
                    for (int k = 0; k < 5; ++k)
                        if (w[3 + k] && prev) {
                            fst[k][g] = (double)(w[3 + k] - prev) * 1e-5;
                            prev = w[3 + k];
                        }
                }
                std::sort(dur.begin(), dur.end());
                std::sort(end.begin(), end.end());
                std::sort(lend.begin(), lend.end());
                fprintf(stderr, "[mrgpu] map workgroups (ms): span %.3f, end min %.3f med %.3f max %.3f, "
                        "main loop end min %.3f med %.3f max %.3f, duration min %.3f med %.3f max %.3f, "
                        "last start %.3f\n", (double)(t1 - t0) * 1e-5, end[0], end[grid / 2], end[grid - 1],
                        lend[0], lend[grid / 2], lend[grid - 1], dur[0], dur[grid / 2], dur[grid - 1],
                        (double)(ls - t0) * 1e-5);
                fprintf(stderr, "[mrgpu] map flush steps (ms, median / max over workgroups):");
                static const char *fn[5] = {"counts", "histogram", "scan", "entries", "totals"};
                for (int k = 0; k < 5; ++k) {
                    std::sort(fst[k].begin(), fst[k].end());
                    fprintf(stderr, " %s %.4f / %.4f", fn[k], fst[k][grid / 2], fst[k][grid - 1]);
                }
                fprintf(stderr, "\n");
            }
        }
        const uint64_t nl = c->h_cnt[CNT_LONG];
        const bool long_full = c->h_cnt[CNT_LONGX] > A.lovf;
        if (c->h_cnt[CNT_OVF] == 0 && !long_full) break;
        if (spec.live) c->st.spec_agg = 2;  // the rerun invalidates the queued aggregation
        agg_put(c, spec);
        // capacity exceeded: grow each bucket's regions to its demand (remembered), run again
        if (c->h_cnt[CNT_OVF]) {
            std::vector<uint32_t> cnt((uint64_t)grid * MRG_NBUCKET), cnt16((uint64_t)grid * MRG_NBUCKET, 0);
            HIPCHK(hipMemcpyAsync(cnt.data(), M.bcount, 4ull * cnt.size(), hipMemcpyDeviceToHost, s));
            if (!idx) HIPCHK(hipMemcpyAsync(cnt16.data(), M.bcount16, 4ull * cnt16.size(), hipMemcpyDeviceToHost, s));
            sync(c);
            c->bcap_rate.assign(MRG_NBUCKET, 0.0);
            c->bcap16_rate.assign(MRG_NBUCKET, 0.0);
            for (int b = 0; b < MRG_NBUCKET; ++b) {
                uint64_t mx = 0, mx16 = 0;
                for (int g = 0; g < grid; ++g) {
                    mx = std::max<uint64_t>(mx, cnt[(uint64_t)g * MRG_NBUCKET + b]);
                    mx16 = std::max<uint64_t>(mx16, cnt16[(uint64_t)g * MRG_NBUCKET + b]);
                }
                bcap[b] = std::max<uint64_t>(bcap[b], mx + mx / 4 + 64);
                c->bcap_rate[b] = (double)mx / per_wg;
                if (!idx) {
                    bcap16[b] = std::max<uint64_t>(bcap16[b], mx16 + mx16 / 4 + 16);
                    c->bcap16_rate[b] = (double)mx16 / per_wg;
                }
            }
            ocap = c->ocap_hint = 4 * ocap;
        }
        if (long_full) {  // a workgroup's long tokens overflowed its region and the list: grow both
            std::vector<uint32_t> lc((uint64_t)grid);
            HIPCHK(hipMemcpyAsync(lc.data(), M.lcount, 4ull * grid, hipMemcpyDeviceToHost, s));
            sync(c);
            const uint64_t mx = *std::max_element(lc.begin(), lc.end());
            c->lper_hint = mx + mx / 4 + 64;
            lcap = c->long_hint = std::max<uint64_t>(lcap, nl + nl / 8 + 1024);
        }
        if (getenv("MRG_DEBUG"))
            fprintf(stderr, "[mrgpu] map rerun: tail overflow %llu, long %llu (list %llu of %llu)\n",
                    (unsigned long long)c->h_cnt[CNT_OVF], (unsigned long long)nl,
                    (unsigned long long)c->h_cnt[CNT_LONGX], (unsigned long long)A.lovf);
        M.release(p);
    }
    if (getenv("MRG_DEBUG"))
        fprintf(stderr, "[mrgpu] map: %llu tokens, %llu tail records, %llu long, %u launches, grid %d\n",
                (unsigned long long)c->h_cnt[CNT_TOKENS], (unsigned long long)c->h_cnt[CNT_REC],
                (unsigned long long)c->h_cnt[CNT_LONG], launches, grid);
    c->st.ms_map = ev_ms(c, 0, 1);
    c->st.map_launches = launches;
    c->st.input_bytes = total;
    c->st.tokens = c->h_cnt[CNT_TOKENS];
    c->st.long_tokens = c->h_cnt[CNT_LONG];
    c->st.map_records = c->h_cnt[CNT_REC];
    c->st.nonascii_tiles = c->h_cnt[CNT_NONASCII];
    c->st.tail_records_16 = is_idx(c) ? 0 : c->h_cnt[CNT_REC16];  // the indexer's are all 24-byte records
    const uint64_t errpos = c->h_cnt[CNT_ERRPOS];
    auto release_map = [&]() {
        agg_put(c, spec);
        M.release(p);
        p.put(d_doc_off); p.put(d_cb); p.put(d_ids);
    };
    if (errpos != ~0ull) {
        release_map();
        uint32_t d = 0;
        while (d + 1 < nd && c->doc_off[d + 1] <= errpos) ++d;
        raise(MRG_EUTF8, "stream did not contain valid UTF-8: document %u (id %u), byte offset %llu", d, ids[d],
              (unsigned long long)(errpos - c->doc_off[d]));
    }
    if (!spec.live) ev_rec(c, 2);
    LongItems li{};
    li.base = c->d_in; li.cnt = nullptr;
    li.n = c->h_cnt[CNT_LONG];
    if (li.n) {  // pack the workgroups' regions and the shared list densely
        M.dstart = pget<uint64_t>(p, li.n);
        M.dlen = pget<uint32_t>(p, li.n);
        M.ddoc = pget<uint32_t>(p, li.n);
        mrg_launch_long_compact(A, grid, M.dstart, M.dlen, M.ddoc, s);
    }
    li.start = M.dstart; li.rawlen = M.dlen; li.doc = M.ddoc;
    // high cardinality (most tokens missed the map-side combine): sort-based aggregation
    bool wide = !idx && c->h_cnt[CNT_REC] > (32ull << 20) && 2 * c->h_cnt[CNT_REC] > c->h_cnt[CNT_TOKENS];
    if (const char *v = getenv("MRG_WIDE")) wide = !idx && atoi(v) != 0;  // test / tuning override
    if (wide && spec.live) {  // the queued aggregation was not needed: its counters back to the map's zeros
        c->st.spec_agg = 2;
        agg_put(c, spec);
        HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_KEYS], 0, 8, s));
        HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_OVF2], 0, 8, s));
    }
    if (wide) c->spec_agg = false;
    if (wide || !bucket_aggregate(c, A, (uint32_t)grid, cap, li, &spec)) {
        c->spec_agg = false;
        c->st.agg_path = 2;
        c->wide_hint = !idx;
        wide_aggregate(c, A, (uint32_t)grid, cap, li);
    }
    ev_rec(c, 3);
    release_map();
    c->st.ms_aggregate = ev_ms(c, 2, 3);
    if (!idx && total >= (64ull << 20)) c->wc_sized = true;
    c->mapped = true;
}

// Indexer document order = bytewise order of the names (the indexer reduce sorts its values):
// rank of each global document id, and the names concatenated in rank order, on the device.
struct DocRank {
    uint32_t *rank = nullptr;
    uint8_t *names = nullptr;
    uint64_t *name_off = nullptr;
    void release(Pool &p) {
        p.put(rank); p.put(names); p.put(name_off);
        *this = DocRank{};
    }
};

DocRank doc_ranks(mrg_ctx *c) {
    DocRank d;
    if (!is_idx(c)) return d;
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint32_t nn = (uint32_t)c->names.size();
    if (nn == 0) raise(MRG_EINVAL, "indexer needs document names (mrg_job_set_doc_names)");
    std::vector<uint32_t> order(nn);
    for (uint32_t i = 0; i < nn; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return c->names[a] < c->names[b]; });
    std::vector<uint32_t> rank(nn);
    std::vector<uint64_t> noff(nn + 1, 0);
    std::string cat;
    for (uint32_t r = 0; r < nn; ++r) {
        rank[order[r]] = r;
        cat += c->names[order[r]];
        noff[r + 1] = cat.size();
    }
    d.rank = pget<uint32_t>(p, nn);
    d.names = pget<uint8_t>(p, cat.size() + 1);
    d.name_off = pget<uint64_t>(p, nn + 1);
    HIPCHK(hipMemcpyAsync(d.rank, rank.data(), 4ull * nn, hipMemcpyHostToDevice, s));
    if (!cat.empty()) HIPCHK(hipMemcpyAsync(d.names, cat.data(), cat.size(), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d.name_off, noff.data(), 8ull * (nn + 1), hipMemcpyHostToDevice, s));
    sync(c);  // host vectors go out of scope
    return d;
}

// Sort records of the keys `ks` by (partition < R, key bytes[, doc rank]) (worker.rs:162-164).
// Returns a or b.  With `defer`, only the MSD passes are enqueued and b is returned: the caller
// checks the oversized-bucket count (c->h_cnt[CNT_N], pinned) after its next stream sync and calls
// mrg_msd_sort_finish if it is not 0 (saves a host round trip per reduce).
SortPlan sort_plan(mrg_ctx *c, uint32_t R) {
    const bool idx = is_idx(c);
    SortPlan plan{};
    plan.use_part = R > 1;
    plan.part_bytes = bytes_for(R - 1);
    plan.use_k0 = plan.use_k1 = true;
    plan.use_doc = idx;
    plan.doc_bytes = idx ? bytes_for(c->names.size() - 1) : 0;
    return plan;
}

SortRec *sort_keys(mrg_ctx *c, KeySet ks, uint32_t R, const uint32_t *d_rank, SortRec *a, SortRec *b, void *stmp,
                   bool defer = false, bool carry = false) {
    const uint64_t n = c->keys.n;
    mrg_launch_make_sortrec(ks, n, d_rank, a, c->stream, carry);
    check_sort_n(n, "key sort");
    const uint32_t pbits = R > 1 ? 32u - (uint32_t)__builtin_clz(R - 1u) : 0u;
    uint32_t *h_nbig = (uint32_t *)&c->h_cnt[CNT_N];
    if (defer) {
        mrg_msd_sort_launch(a, b, n, pbits, stmp, c->stream, h_nbig);
        return n <= 1 ? a : b;
    }
    uint32_t n_big = 0;
    return mrg_msd_sort(a, b, n, pbits, sort_plan(c, R), stmp, c->stream, &n_big, h_nbig);
}

FormatArgs format_args(mrg_ctx *c, const SortRec *recs, KeySet ks, uint32_t R, int drop_last, const DocRank &dr,
                       bool carried = false) {
    FormatArgs f{};
    f.carried = carried ? 1 : 0;
    f.recs = recs;
    f.n = c->keys.n;
    f.ks = ks;
    f.heap = c->keys.heap;
    f.heap_bytes = c->keys.heap_bytes;
    f.n_reduce = R;
    f.drop_last = drop_last;
    f.indexer = is_idx(c);
    f.any_long = c->keys.any_long;
    f.names = dr.names;
    f.name_off = dr.name_off;
    return f;
}

int compat_drop_last(const mrg_ctx *c) { return (c->flags & MRG_FLAG_NO_COMPAT_DROP_LAST) ? 0 : 1; }

// mr-{r}.txt of a wide result straight from its leaves (k_wide.hip): last-group drop on the last
// non-empty leaf of every partition, a scan of the leaf byte totals, the line writer.
void wide_reduce(mrg_ctx *c) {
    WideRes &w = c->wide;
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint64_t NL = (uint64_t)w.B1 * MRG_WIDE_MAXB2;
    ev_rec(c, 4);
    uint32_t *drop = pget<uint32_t>(p, NL);
    HIPCHK(hipMemsetAsync(drop, 0, 4 * NL, s));
    uint64_t *bytes = pget<uint64_t>(p, NL + 1), *off = pget<uint64_t>(p, NL + 1);
    uint64_t *tmp = pget<uint64_t>(p, mrg_scan_tmp_elems(NL + 1));
    HIPCHK(hipMemcpyAsync(bytes, w.leaf_bytes, 8 * (NL + 1), hipMemcpyDeviceToDevice, s));
    if (compat_drop_last(c)) mrg_wide_launch_drop(w.nleaf, w.B1r, c->R, w.leaf_nd, bytes, w.leaf_last, drop, s);
    mrg_scan_u64(bytes, off, NL + 1, tmp, s);  // off[NL] = total (bytes[NL] == 0)
    uint64_t total = 0;
    HIPCHK(hipMemcpyAsync(&total, off + NL, 8, hipMemcpyDeviceToHost, s));
    sync(c);
    ev_rec(c, 5);
    if (total + 16 > c->out_cap) {
        if (c->d_out) p.put(c->d_out);
        c->out_cap = total + 16;
        c->d_out = pget<uint8_t>(p, c->out_cap);
    }
    if (getenv("MRG_DEBUG_FILL_OUT")) HIPCHK(hipMemsetAsync(c->d_out, 0xEE, total, s));  // diagnostics: unwritten bytes show
    mrg_wide_launch_write(w.kout, w.ocnt, w.leaf_pk, w.nleaf, w.leaf_out, w.leaf_nd, drop, off, w.B1, c->d_out, s);
    uint64_t *poff = pget<uint64_t>(p, c->R + 1);
    mrg_wide_launch_part_off(off, w.B1r, c->R, total, poff, s);
    c->part_off.assign(c->R + 1, 0);
    HIPCHK(hipMemcpyAsync(c->part_off.data(), poff, 8ull * (c->R + 1), hipMemcpyDeviceToHost, s));
    ev_rec(c, 6);
    sync(c);
    HIPCHK(hipGetLastError());
    p.put(drop); p.put(bytes); p.put(off); p.put(tmp); p.put(poff);
    c->out_bytes = total;
    c->st.ms_sort = ev_ms(c, 4, 5);
    c->st.ms_format = ev_ms(c, 5, 6);
    c->st.output_bytes = total;
    c->reduced = true;
}

void job_reduce(mrg_ctx *c) {
    need_job(c);
    if (!c->mapped) raise(MRG_EINVAL, "nothing to reduce: call mrg_job_map or mrg_job_import first");
    if (c->wide.ready) {
        wide_reduce(c);
        return;
    }
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint64_t n = c->keys.n;
    DocRank dr = doc_ranks(c);
    ev_rec(c, 4);
    SortRec *a = pget<SortRec>(p, n), *b = pget<SortRec>(p, n);
    void *stmp = p.get(mrg_sort_tmp_bytes(n));
    SortRec *sorted = a;
    const bool presorted = c->keys.sorted && !c->keys.any_long && !is_idx(c);
    // the oversized-bucket check of the key sort waits for format's own sync (add_first below is
    // not idempotent: that path checks at once)
    const bool defer = !presorted && !(c->extra_first && n);
    // wc: counts and lengths carried in the sort records, unless the text reduce's empty-key quirk
    // adds to the first key's count after the sort
    const bool carry = !is_idx(c) && !c->extra_first;
    if (presorted) mrg_launch_make_sortrec(c->keys.ks, n, nullptr, a, s, carry);
    else sorted = sort_keys(c, c->keys.ks, c->R, dr.rank, a, b, stmp, defer, carry);
    // text reduce (worker.rs:169-173): lines with an empty key sort first and, since `prev` is still
    // empty when the first real key arrives, their values join that key's group
    if (c->extra_first && n) {
        if (c->keys.any_long) mrg_launch_fix_runs(sorted, n, c->keys.ks, c->keys.heap, s);
        mrg_launch_add_first(sorted, c->keys.ks, c->extra_first, s);
    }
    ev_rec(c, 5);
    const FormatArgs f = format_args(c, sorted, c->keys.ks, c->R, compat_drop_last(c), dr, carry);
    c->part_off.assign(c->R + 1, 0);
    c->out_bytes = mrg_format(f, p, &c->d_out, &c->out_cap, c->part_off.data(), s);
    const uint32_t n_big = *(const uint32_t *)&c->h_cnt[CNT_N];  // written by the sort's async copy
    if (defer && n > 1 && n_big) {  // oversized MSD buckets: sort them, format again
        sorted = mrg_msd_sort_finish(a, b, n, sort_plan(c, c->R), stmp, s, n_big);
        const FormatArgs f2 = format_args(c, sorted, c->keys.ks, c->R, compat_drop_last(c), dr, carry);
        c->out_bytes = mrg_format(f2, p, &c->d_out, &c->out_cap, c->part_off.data(), s);
    }
    ev_rec(c, 6);
    HIPCHK(hipGetLastError());
    p.put(a); p.put(b); p.put(stmp);
    dr.release(p);
    c->st.ms_sort = ev_ms(c, 4, 5);
    c->st.ms_format = ev_ms(c, 5, 6);
    c->st.output_bytes = c->out_bytes;
    c->reduced = true;
}

// final.txt (src/run.sh:16-20 with LC_ALL=C): the lines of every partition this context holds,
// sorted bytewise, written on the device.  The keys the per-partition pass drops (drop-last) are
// found in the partition order, moved to a second "partition" and the rest re-sorted by key alone.
void job_final(mrg_ctx *c) {
    need_job(c);
    if (!c->mapped) raise(MRG_EINVAL, "no keys: call mrg_job_map or mrg_job_import first");
    wide_densify(c, 0);
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint64_t n = c->keys.n;
    DocRank dr = doc_ranks(c);
    SortRec *a = pget<SortRec>(p, n), *b = pget<SortRec>(p, n);
    void *stmp = p.get(mrg_sort_tmp_bytes(n));
    const int drop = compat_drop_last(c);
    uint32_t *part2 = pget<uint32_t>(p, std::max<uint64_t>(n, 1));
    KeySet ks2 = c->keys.ks;
    ks2.part = part2;
    if (drop) {
        SortRec *s1 = sort_keys(c, c->keys.ks, c->R, dr.rank, a, b, stmp);
        if (c->keys.any_long) mrg_launch_fix_runs(s1, n, c->keys.ks, c->keys.heap, s);
        mrg_launch_final_part(s1, n, c->keys.ks, c->keys.heap, drop, part2, s);
    } else {
        mrg_launch_fill_u32(part2, 0u, n, s);
    }
    const uint32_t R2 = drop ? 2u : 1u;
    SortRec *s2 = sort_keys(c, ks2, R2, dr.rank, a, b, stmp);
    const FormatArgs f = format_args(c, s2, ks2, R2, 0, dr);
    uint64_t po[3] = {0, 0, 0};
    mrg_format(f, p, &c->d_final, &c->final_cap, po, s);
    HIPCHK(hipGetLastError());
    p.put(a); p.put(b); p.put(stmp); p.put(part2);
    dr.release(p);
    c->final_bytes = po[1];
    c->finalized = true;
}

void export_sizes(mrg_ctx *c, uint32_t n_owners, uint64_t *h_rec, uint64_t *h_heap) {
    need_job(c);
    if (!c->mapped) raise(MRG_EINVAL, "export before map");
    if (n_owners == 0) raise(MRG_EINVAL, "n_owners must be > 0");
    wide_densify(c, 0);
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    unsigned long long *d = pget<unsigned long long>(p, 2ull * n_owners);
    HIPCHK(hipMemsetAsync(d, 0, 16ull * n_owners, s));
    c->xrec_vmax = std::max<uint64_t>(1, std::min<uint64_t>(MRG_XREC_VMAX, env_u64("MRG_TEST_XREC_VMAX", MRG_XREC_VMAX)));
    mrg_launch_export_count(c->keys.ks, c->keys.n, n_owners, d, d + n_owners, is_idx(c), c->xrec_vmax, s);
    std::vector<uint64_t> h(2ull * n_owners);
    HIPCHK(hipMemcpyAsync(h.data(), d, 16ull * n_owners, hipMemcpyDeviceToHost, s));
    sync(c);
    p.put(d);
    c->n_owners = n_owners;
    c->exp_rec.assign(h.begin(), h.begin() + n_owners);
    c->exp_heap.assign(h.begin() + n_owners, h.end());
    if (h_rec) memcpy(h_rec, c->exp_rec.data(), 8ull * n_owners);
    if (h_heap) memcpy(h_heap, c->exp_heap.data(), 8ull * n_owners);
}

// wait = false: the caller consumes the packed records on the context's stream (the library's own
// exchange): no host wait here
void export_pack(mrg_ctx *c, void *d_rec, void *d_heap, bool wait = true) {
    need_job(c);
    if (!c->n_owners) raise(MRG_EINVAL, "call mrg_job_export_sizes first");
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint32_t G = c->n_owners;
    std::vector<uint64_t> base(2ull * G, 0);
    for (uint32_t o = 1; o < G; ++o) {
        base[o] = base[o - 1] + c->exp_rec[o - 1];
        base[G + o] = base[G + o - 1] + c->exp_heap[o - 1];
    }
    uint64_t *d_base = pget<uint64_t>(p, 2ull * G);
    unsigned long long *cur = pget<unsigned long long>(p, 2ull * G);
    HIPCHK(hipMemcpyAsync(d_base, base.data(), 16ull * G, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(cur, 0, 16ull * G, s));
    mrg_launch_export_pack(c->keys.ks, c->keys.heap, c->keys.n, G, d_base, d_base + G, cur, cur + G, (XRec *)d_rec,
                           (uint8_t *)d_heap, is_idx(c), c->xrec_vmax, s);
    if (wait) sync(c);
    p.put(d_base);  // later users of these blocks run after the pack on the same stream
    p.put(cur);
}

// Received records -> the job's keys: exchange records (xr, include/mrgpu.h) or the text reduce's
// line records (lr, k_text.hip).
void import_recs(mrg_ctx *c, const XRec *xr, const LRec *lr, uint64_t n_rec, const void *d_heap, uint64_t heap_bytes,
                 const uint64_t *seg_recs, const uint64_t *seg_heap, uint32_t n_segs) {
    need_job(c);
    c->wide.release(c->pool);  // the imported records replace the job's keys, whatever path the map took
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    std::vector<uint64_t> rec_end, heap_base;
    if (n_segs == 0) {
        rec_end.push_back(n_rec);
        heap_base.push_back(0);
        n_segs = 1;
    } else {
        uint64_t r = 0, h = 0;
        for (uint32_t i = 0; i < n_segs; ++i) {
            heap_base.push_back(h);
            r += seg_recs[i];
            h += seg_heap[i];
            rec_end.push_back(r);
        }
        if (r != n_rec || h != heap_bytes) raise(MRG_EINVAL, "segment sizes do not add up to n_rec / heap_bytes");
    }
    uint64_t *d_seg = pget<uint64_t>(p, 2ull * n_segs);
    HIPCHK(hipMemcpyAsync(d_seg, rec_end.data(), 8ull * n_segs, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_seg + n_segs, heap_base.data(), 8ull * n_segs, hipMemcpyHostToDevice, s));
    LongItems li{};
    li.base = (const uint8_t *)d_heap;
    li.start = pget<uint64_t>(p, n_rec);
    li.rawlen = pget<uint32_t>(p, n_rec);
    li.doc = pget<uint32_t>(p, n_rec);
    li.cnt = pget<uint64_t>(p, n_rec);
    li.verbatim = 1;  // the exchange heap holds exact key bytes
    HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_LONG], 0, 8, s));
    if (xr) mrg_launch_x_split_long(xr, n_rec, d_seg, d_seg + n_segs, n_segs, li, &c->d_cnt[CNT_LONG], is_idx(c), s);
    else mrg_launch_l_split_long(lr, n_rec, d_seg, d_seg + n_segs, n_segs, li, &c->d_cnt[CNT_LONG], s);
    read_counters(c);
    li.n = c->h_cnt[CNT_LONG];
    ShortSrc src;
    src.x = xr;
    src.lx = lr;
    src.n = n_rec;
    ev_rec(c, 2);
    aggregate(c, src, li);
    ev_rec(c, 3);
    sync(c);
    p.put(d_seg); p.put(li.start); p.put(li.rawlen); p.put(li.doc); p.put(li.cnt);
    c->st.ms_aggregate = ev_ms(c, 2, 3);
    c->mapped = true;
    c->reduced = false;
}

void job_import(mrg_ctx *c, const void *d_rec, uint64_t n_rec, const void *d_heap, uint64_t heap_bytes,
                const uint64_t *seg_recs, const uint64_t *seg_heap, uint32_t n_segs) {
    import_recs(c, (const XRec *)d_rec, nullptr, n_rec, d_heap, heap_bytes, seg_recs, seg_heap, n_segs);
}

// A communicator shell with its preallocated exchange buffers (the RCCL communicator is added by
// the caller).
mrg_comm *comm_alloc(int device, int n, int rank) {
    HIPCHK(hipSetDevice(device));
    mrg_comm *m = new mrg_comm();
    m->n = n;
    m->rank = rank;
    m->device = device;
    if (hipMalloc(&m->d_counts, 48ull * (uint64_t)n) != hipSuccess || hipMalloc(&m->d_flag, 64) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFree(m->d_counts);
        delete m;
        raise(MRG_ENOMEM, "communicator buffers: device allocation failed");
    }
    return m;
}

void comm_free(mrg_comm *m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    (void)hipFree(m->d_counts);
    (void)hipFree(m->d_flag);
    delete m;
}

// Test knob: MRG_TEST_FAIL="<stage>[:<rank>]" raises an injected failure at that stage (on that rank
// only, or on every rank), so the failure paths of the multi-GPU plan can be exercised.
void test_fail(const char *stage, int rank) {
    const char *v = getenv("MRG_TEST_FAIL");
    if (!v || !*v) return;
    const char *colon = strchr(v, ':');
    const size_t n = colon ? (size_t)(colon - v) : strlen(v);
    if (n == strlen(stage) && !strncmp(v, stage, n) && (!colon || atoi(colon + 1) == rank))
        raise(MRG_EINVAL, "injected failure at stage '%s' on rank %d (MRG_TEST_FAIL)", stage, rank);
}

// An RCCL call of the exchange: on failure the communicator is aborted (its peers' pending operations
// then fail instead of waiting forever) and the call raises MRG_ECOMM.
// Caller holds m->mu (a CommLock).
void nccl_or_abort(mrg_comm *m, ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return;
    if (!m->aborted.exchange(true)) (void)ncclCommAbort(m->comm);
    raise(MRG_ECOMM, "%s: %s (communicator aborted)", what, ncclGetErrorString(r));
}

void check_not_aborted(mrg_comm *m) {
    if (m->aborted.load()) raise(MRG_ECOMM, "the communicator was aborted (another rank of the job failed)");
}

// The communicator's lock for a run of RCCL enqueues, taken only if it has not been aborted (the
// abort frees it): a watchdog abort waits for the enqueues, and enqueues after it raise MRG_ECOMM.
struct CommLock {
    std::unique_lock<std::timed_mutex> lk;
    explicit CommLock(mrg_comm *m) : lk(m->mu) { check_not_aborted(m); }
};

// Abort from any thread (mrg_run_job's watchdog), serialised with the rank threads' enqueues until
// `deadline`.  An enqueue can itself block inside RCCL (a first send/recv to a peer sets up the
// connection and waits for that peer): a lock still held at the deadline belongs to such a blocked
// call, and the abort then goes ahead without the lock -- the accepted exception to the lock's rule,
// since releasing a blocked call is exactly what ncclCommAbort exists for.  The watchdog aborts all
// ranks in parallel against one deadline (a job with G hung ranks waits once, not G times).
void comm_abort(mrg_comm *m, std::chrono::steady_clock::time_point deadline) {
    std::unique_lock<std::timed_mutex> lk(m->mu, std::defer_lock);
    (void)lk.try_lock_until(deadline);
    if (m->comm && !m->aborted.exchange(true)) (void)ncclCommAbort(m->comm);
}

// Max of `flag` over the ranks (one RCCL all-reduce into the preallocated status word): every rank
// learns whether any rank failed, so all of them leave the exchange together.
int agree(mrg_ctx *c, mrg_comm *m, int flag) {
    check_not_aborted(m);
    HIPCHK(hipMemcpyAsync(m->d_flag, &flag, sizeof flag, hipMemcpyHostToDevice, c->stream));
    {
        CommLock lk(m);
        nccl_or_abort(m, ncclAllReduce(m->d_flag, m->d_flag, 1, ncclInt, ncclMax, m->comm, c->stream), "ncclAllReduce");
    }
    int any = 0;
    HIPCHK(hipMemcpyAsync(&any, m->d_flag, sizeof any, hipMemcpyDeviceToHost, c->stream));
    sync(c);
    check_not_aborted(m);
    return any;
}

// The shuffle: the reference's map -> reduce hand-off through mr-{m}-{r}.txt files
// (worker.rs:117-140 -> 79-109) as one exchange over RCCL.  Owner of partition r = r % G.
//
// Failure protocol: every rank reaches every collective of the exchange.  A rank whose local step
// fails (export, buffer allocation) still takes part, with a failure status: the per-destination
// counts message carries it (the first collective), and one status all-reduce precedes the data
// transfer; every rank then raises together (the failing rank its own error, the others MRG_ECOMM).
// An RCCL error aborts the communicator.
// Pool buffers of one exchange, returned to the pool on every exit (a failed collective or a watchdog
// abort throws past the success path).
struct PoolLease {
    Pool &p;
    uint8_t *b[4] = {nullptr, nullptr, nullptr, nullptr};
    explicit PoolLease(Pool &pool) : p(pool) {}
    PoolLease(const PoolLease &) = delete;
    PoolLease &operator=(const PoolLease &) = delete;
    uint8_t *get(int i, uint64_t bytes) { return b[i] = pget<uint8_t>(p, bytes); }
    void put(int i) {
        p.put(b[i]);
        b[i] = nullptr;
    }
    ~PoolLease() {
        for (int i = 0; i < 4; ++i) p.put(b[i]);
    }
};

// A pair of timing events, destroyed on every exit.
struct EventPair {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    EventPair() {
        HIPCHK(hipEventCreate(&e0));
        if (hipEventCreate(&e1) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipEventDestroy(e0);
            raise(MRG_EHIP, "hipEventCreate failed");
        }
    }
    EventPair(const EventPair &) = delete;
    EventPair &operator=(const EventPair &) = delete;
    ~EventPair() {
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
};

// An RCCL call inside the send/recv group: on failure the group is closed first (the calling thread's
// group depth stays balanced for its next RCCL call), then the communicator is aborted.
void group_or_abort(mrg_comm *m, ncclResult_t r, const char *what) {
    if (r == ncclSuccess) return;
    (void)ncclGroupEnd();
    nccl_or_abort(m, r, what);
}

void job_shuffle(mrg_ctx *c, mrg_comm *m) {
    if (!c || !m || !m->comm) raise(MRG_EINVAL, "null context or communicator");
    if (m->device != c->device) raise(MRG_EINVAL, "communicator is on device %d, context on %d", m->device, c->device);
    check_not_aborted(m);
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    const uint32_t G = (uint32_t)m->n;
    const uint32_t me = (uint32_t)m->rank;
    const uint64_t X = MRG_XREC_BYTES;
    enum { SREC, SHEAP, RREC, RHEAP };
    PoolLease buf(p);  // send records / heap, receive records / heap: returned on every exit
    MrgError mine{MRG_OK, ""};
    // ---- local: export sizes and pack (the pack runs on the stream, no host wait)
    std::vector<uint64_t> sc(3ull * G, 0), rc(3ull * G, 0);  // per peer: records, heap bytes, status
    std::vector<uint64_t> sro(G + 1, 0), sho(G + 1, 0);
    try {
        need_job(c);
        if (!c->mapped) raise(MRG_EINVAL, "shuffle before map");
        test_fail("export", (int)me);
        export_sizes(c, G, nullptr, nullptr);
        for (uint32_t o = 0; o < G; ++o) {
            sc[3 * o] = c->exp_rec[o];
            sc[3 * o + 1] = c->exp_heap[o];
            sro[o + 1] = sro[o] + sc[3 * o];
            sho[o + 1] = sho[o] + sc[3 * o + 1];
        }
        buf.get(SREC, sro[G] * X + 16);
        buf.get(SHEAP, sho[G] + 16);
        export_pack(c, buf.b[SREC], buf.b[SHEAP], false);
    } catch (const MrgError &e) {
        mine = e;
        std::fill(sc.begin(), sc.end(), 0);
    }
    uint8_t *const srec = buf.b[SREC], *const sheap = buf.b[SHEAP];
    for (uint32_t o = 0; o < G; ++o) sc[3 * o + 2] = mine.code ? 1u : 0u;
    // ---- collective 1: the counts all-to-all (with every rank's status)
    HIPCHK(hipMemcpyAsync(m->d_counts, sc.data(), 24ull * G, hipMemcpyHostToDevice, s));
    {
        CommLock lk(m);
        nccl_or_abort(m, ncclAllToAll(m->d_counts, m->d_counts + 3 * G, 3, ncclUint64, m->comm, s), "ncclAllToAll");
    }
    HIPCHK(hipMemcpyAsync(rc.data(), m->d_counts + 3 * G, 24ull * G, hipMemcpyDeviceToHost, s));
    sync(c);
    check_not_aborted(m);
    int failed_peer = -1;
    for (uint32_t o = 0; o < G; ++o)
        if (rc[3 * o + 2] && failed_peer < 0) failed_peer = (int)o;
    if (mine.code) throw mine;
    if (failed_peer >= 0) raise(MRG_ECOMM, "rank %d of the exchange failed before sending", failed_peer);
    // ---- local: receive buffers
    std::vector<uint64_t> rro(G + 1, 0), rho(G + 1, 0), seg_rec(G), seg_heap(G);
    for (uint32_t o = 0; o < G; ++o) {
        rro[o + 1] = rro[o] + rc[3 * o];
        rho[o + 1] = rho[o] + rc[3 * o + 1];
        seg_rec[o] = rc[3 * o];
        seg_heap[o] = rc[3 * o + 1];
    }
    try {
        test_fail("recv", (int)me);
        buf.get(RREC, rro[G] * X + 16);
        buf.get(RHEAP, rho[G] + 16);
    } catch (const MrgError &e) {
        mine = e;
    }
    // ---- collective 2: everyone ready to transfer?
    if (agree(c, m, mine.code ? 1 : 0)) {
        if (mine.code) throw mine;
        raise(MRG_ECOMM, "another rank of the exchange could not allocate its receive buffers");
    }
    uint8_t *const rrec = buf.b[RREC], *const rheap = buf.b[RHEAP];
    // ---- collective 3: own slice by a device copy; peers by one send/recv group (each peer pair has
    // its own xGMI link)
    EventPair ev;
    HIPCHK(hipEventRecord(ev.e0, s));
    if (sc[3 * me]) HIPCHK(hipMemcpyAsync(rrec + rro[me] * X, srec + sro[me] * X, sc[3 * me] * X, hipMemcpyDeviceToDevice, s));
    if (sc[3 * me + 1]) HIPCHK(hipMemcpyAsync(rheap + rho[me], sheap + sho[me], sc[3 * me + 1], hipMemcpyDeviceToDevice, s));
    uint64_t sent = 0, recv = 0;
    {
        CommLock lk(m);
        nccl_or_abort(m, ncclGroupStart(), "ncclGroupStart");
        // test knob: an RCCL failure inside the group, after the events and all four buffers exist
        if (getenv("MRG_TEST_FAIL")) {
            try {
                test_fail("sendrecv", (int)me);
            } catch (const MrgError &) {
                group_or_abort(m, ncclInternalError, "ncclSend (MRG_TEST_FAIL=sendrecv)");
            }
        }
        for (uint32_t o = 0; o < G; ++o) {
            if (o == me) continue;
            if (sc[3 * o]) group_or_abort(m, ncclSend(srec + sro[o] * X, sc[3 * o] * X, ncclUint8, (int)o, m->comm, s), "ncclSend");
            if (sc[3 * o + 1]) group_or_abort(m, ncclSend(sheap + sho[o], sc[3 * o + 1], ncclUint8, (int)o, m->comm, s), "ncclSend");
            if (rc[3 * o]) group_or_abort(m, ncclRecv(rrec + rro[o] * X, rc[3 * o] * X, ncclUint8, (int)o, m->comm, s), "ncclRecv");
            if (rc[3 * o + 1]) group_or_abort(m, ncclRecv(rheap + rho[o], rc[3 * o + 1], ncclUint8, (int)o, m->comm, s), "ncclRecv");
            sent += sc[3 * o] * X + sc[3 * o + 1];
            recv += rc[3 * o] * X + rc[3 * o + 1];
        }
        nccl_or_abort(m, ncclGroupEnd(), "ncclGroupEnd");
    }
    HIPCHK(hipEventRecord(ev.e1, s));
    HIPCHK(hipEventSynchronize(ev.e1));
    check_not_aborted(m);  // a watchdog abort ends a transfer early: its buffers are not to be used
    buf.put(SREC);
    buf.put(SHEAP);
    // ---- local: re-aggregate what arrived (no collective after this point)
    const mrg_stats keep = c->st;
    job_import(c, rrec, rro[G], rheap, rho[G], seg_rec.data(), seg_heap.data(), G);  // ends with a host wait
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ev.e0, ev.e1));
    // the import's aggregation time is the reduce side's; the map-side stats stay those of the map
    const double agg_import = c->st.ms_aggregate;
    c->st = keep;
    c->st.ms_aggregate += agg_import;
    c->st.distinct_keys = c->keys.n;
    c->st.ms_exchange = ms;
    c->st.exchange_sent = sent;
    c->st.exchange_recv = recv;
}

void check_names(const char *const *names, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i) {
        if (!names[i]) raise(MRG_EINVAL, "null document name %u", i);
        for (const char *q = names[i]; *q; ++q)
            if (*q == ' ' || *q == ',' || *q == '\n')
                raise(MRG_EINVAL, "document name '%s' contains ' ', ',' or newline", names[i]);
    }
}

}  // namespace

// ===================================================================== C ABI

// ---- text intermediates: the reference's mr-{m}-{r}.txt, byte for byte

// One map task's intermediates: "key 1\n" per token in input order, partition by SipHash % R
// (worker.rs:117-140).  out = the R files' bytes concatenated, off[R + 1] their offsets.
void text_map(mrg_ctx *c, const uint8_t *h, uint64_t n, uint32_t R, std::vector<uint8_t> &out,
              std::vector<uint64_t> &off) {
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    uint8_t *d = pget<uint8_t>(p, n + 64);
    if (n) HIPCHK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
    const uint64_t nseg = mrg_text_segments(n);
    uint64_t *cnt = pget<uint64_t>(p, nseg + 1), *base = pget<uint64_t>(p, nseg + 1);
    uint64_t *stmp = pget<uint64_t>(p, mrg_scan_tmp_elems(nseg + 1));
    HIPCHK(hipMemsetAsync(cnt, 0, 8 * (nseg + 1), s));
    HIPCHK(hipMemsetAsync(&c->d_cnt[CNT_ERRPOS], 0xFF, 8, s));
    mrg_launch_text_tok(d, n, R, nullptr, cnt, nullptr, &c->d_cnt[CNT_ERRPOS], s);
    mrg_scan_u64(cnt, base, nseg + 1, stmp, s);
    uint64_t T = 0;
    HIPCHK(hipMemcpyAsync(&T, base + nseg, 8, hipMemcpyDeviceToHost, s));
    read_counters(c);
    auto done = [&]() { p.put(d); p.put(cnt); p.put(base); p.put(stmp); };
    if (c->h_cnt[CNT_ERRPOS] != ~0ull) {
        done();
        raise(MRG_EUTF8, "stream did not contain valid UTF-8: byte offset %llu", (unsigned long long)c->h_cnt[CNT_ERRPOS]);
    }
    off.assign(R + 1, 0);
    out.clear();
    if (T) {
        TextTok *tok = pget<TextTok>(p, T);
        mrg_launch_text_tok(d, n, R, base, cnt, tok, &c->d_cnt[CNT_ERRPOS], s);
        uint64_t *part = pget<uint64_t>(p, T), *kv = pget<uint64_t>(p, 4 * T);
        uint32_t *idx = pget<uint32_t>(p, T);
        void *stmp2 = p.get(mrg_sort_tmp_bytes(T));
        mrg_launch_text_keys(tok, T, part, idx, s);
        check_sort_n(T, "text partition sort");
        mrg_radix_sort_u64(part, idx, kv, T, stmp2, s);  // stable: input order inside a partition
        uint64_t *L = pget<uint64_t>(p, T + 1), *O = pget<uint64_t>(p, T + 1);
        uint64_t *stmp3 = pget<uint64_t>(p, mrg_scan_tmp_elems(T + 1));
        mrg_launch_text_len(tok, idx, T, L, s);
        mrg_scan_u64(L, O, T, stmp3, s);
        uint64_t last[2];
        HIPCHK(hipMemcpyAsync(&last[0], O + (T - 1), 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(&last[1], L + (T - 1), 8, hipMemcpyDeviceToHost, s));
        sync(c);
        const uint64_t total = last[0] + last[1];
        uint8_t *ob = pget<uint8_t>(p, total + 16);
        uint64_t *doff = pget<uint64_t>(p, R + 1);
        mrg_launch_text_write(d, tok, idx, T, O, ob, s);
        mrg_launch_text_part_off(part, O, T, R, total, doff, s);
        out.resize(total);
        HIPCHK(hipMemcpyAsync(out.data(), ob, total, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(off.data(), doff, 8ull * (R + 1), hipMemcpyDeviceToHost, s));
        sync(c);
        p.put(tok); p.put(part); p.put(kv); p.put(idx); p.put(stmp2); p.put(L); p.put(O); p.put(stmp3);
        p.put(ob); p.put(doff);
    }
    done();
}

// One reduce task from text intermediates (worker.rs:79-109, 157-193): returns mr-{r}.txt.
void text_reduce(mrg_ctx *c, const uint8_t *const *files, const uint64_t *sizes, size_t k, uint32_t flags,
                 std::vector<uint8_t> &out) {
    job_begin(c, MRG_APP_WC, 1, flags);  // every key read goes to the one output file
    Pool &p = c->pool;
    hipStream_t s = c->stream;
    std::vector<uint64_t> fo(k + 1, 0), fe(k);
    for (size_t i = 0; i < k; ++i) {
        fe[i] = fo[i] + sizes[i];
        fo[i + 1] = (fe[i] + 63) & ~63ull;  // files on 64-byte boundaries (one file per segment)
    }
    const uint64_t total = fo[k];
    uint8_t *d = pget<uint8_t>(p, total + 64);
    HIPCHK(hipMemsetAsync(d, 0, total + 64, s));
    for (size_t i = 0; i < k; ++i)
        if (sizes[i]) HIPCHK(hipMemcpyAsync(d + fo[i], files[i], sizes[i], hipMemcpyHostToDevice, s));
    const uint32_t nf = (uint32_t)std::max<size_t>(k, 1);
    uint64_t *dfo = pget<uint64_t>(p, nf + 1), *dfe = pget<uint64_t>(p, nf);
    if (k) {
        HIPCHK(hipMemcpyAsync(dfo, fo.data(), 8 * k, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(dfe, fe.data(), 8 * k, hipMemcpyHostToDevice, s));
    }
    unsigned long long *err = pget<unsigned long long>(p, 3);  // [utf8 pos, format pos, empty-key lines]
    HIPCHK(hipMemsetAsync(err, 0xFF, 16, s));
    HIPCHK(hipMemsetAsync(err + 2, 0, 8, s));
    mrg_launch_utf8_check(d, total, err, s);  // read_to_string (worker.rs:93); zero padding is valid
    const uint64_t nseg = total / 64;
    uint64_t *cnt = pget<uint64_t>(p, nseg + 1), *base = pget<uint64_t>(p, nseg + 1);
    uint64_t *stmp = pget<uint64_t>(p, mrg_scan_tmp_elems(nseg + 1));
    HIPCHK(hipMemsetAsync(cnt, 0, 8 * (nseg + 1), s));
    if (k) mrg_launch_text_lines(d, dfo, dfe, nf, nseg, nullptr, cnt, nullptr, err, err + 2, s);
    mrg_scan_u64(cnt, base, nseg + 1, stmp, s);
    std::vector<uint64_t> fb(k + 1, 0);  // records before file i = base[fo[i] / 64]
    for (size_t i = 0; i <= k; ++i) HIPCHK(hipMemcpyAsync(&fb[i], base + fo[i] / 64, 8, hipMemcpyDeviceToHost, s));
    unsigned long long herr[3];
    HIPCHK(hipMemcpyAsync(herr, err, sizeof herr, hipMemcpyDeviceToHost, s));
    sync(c);
    auto done = [&]() { p.put(d); p.put(dfo); p.put(dfe); p.put(err); p.put(cnt); p.put(base); p.put(stmp); };
    auto where = [&](uint64_t pos, uint64_t &f) {
        f = 0;
        while (f + 1 < k && fo[f + 1] <= pos) ++f;
        return pos - fo[f];
    };
    if (herr[0] != ~0ull) {
        uint64_t f;
        const uint64_t at = where(herr[0], f);
        done();
        raise(MRG_EUTF8, "intermediate file %llu is not valid UTF-8 (byte offset %llu)", (unsigned long long)f,
              (unsigned long long)at);
    }
    if (herr[1] != ~0ull) {
        uint64_t f;
        const uint64_t at = where(herr[1], f);
        done();
        raise(MRG_EINVAL, "intermediate file %llu: the line at byte %llu does not split into `key value` "
              "(worker.rs:100 asserts two space-separated fields; keys hold no NUL)", (unsigned long long)f,
              (unsigned long long)at);
    }
    const uint64_t N = fb[k];
    LRec *x = pget<LRec>(p, std::max<uint64_t>(N, 1));
    if (k) mrg_launch_text_lines(d, dfo, dfe, nf, nseg, base, cnt, x, err, err + 2, s);  // also counts empty keys
    HIPCHK(hipMemcpyAsync(&herr[2], err + 2, 8, hipMemcpyDeviceToHost, s));
    sync(c);
    std::vector<uint64_t> seg_rec(nf, 0), seg_heap(nf, 0);
    for (size_t i = 0; i < k; ++i) {
        seg_rec[i] = fb[i + 1] - fb[i];
        seg_heap[i] = fo[i + 1] - fo[i];  // heap segment of file i = its slot in the buffer
    }
    import_recs(c, nullptr, x, N, d, k ? total : 0, seg_rec.data(), seg_heap.data(), nf);
    c->extra_first = herr[2];
    job_reduce(c);
    out.resize(c->out_bytes);
    if (c->out_bytes) HIPCHK(hipMemcpyAsync(out.data(), c->d_out, c->out_bytes, hipMemcpyDeviceToHost, s));
    sync(c);
    if (c->keys.n == 0 && herr[2] && (flags & MRG_FLAG_NO_COMPAT_DROP_LAST)) {  // only empty keys, group kept
        const std::string line = " " + std::to_string(herr[2]) + "\n";
        out.assign(line.begin(), line.end());
    }
    p.put(x);
    done();
}

extern "C" {

const char *mrg_last_error(void) { return g_err.c_str(); }
const char *mrg_version(void) { return "mrgpu 0.6 (gfx950, abi 6)"; }

int mrg_open(int device, mrg_ctx **out) {
    return guard([&] {
        if (!out) raise(MRG_EINVAL, "null out");
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        if (device < 0 || device >= ndev) raise(MRG_EINVAL, "device %d not present (%d devices)", device, ndev);
        HIPCHK(hipSetDevice(device));
        mrg_ctx *c = new mrg_ctx();
        c->device = device;
        c->pool.set_device(device);
        HIPCHK(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
        c->stream = c->own;
        HIPCHK(hipMalloc(&c->d_cnt, sizeof(unsigned long long) * CNT_N));
        // CNT_N counters + pinned scratch (h_cnt[CNT_N]: the key sort's oversized-bucket count)
        // [CNT_N, CNT_N + 8): scratch; [CNT_N + 8, + MRG_NBUCKET / 2): the map's overflow-list fill (u32)
        HIPCHK(hipHostMalloc(&c->h_cnt, sizeof(unsigned long long) * (CNT_N + 8 + MRG_NBUCKET / 2), hipHostMallocDefault));
        HIPCHK(hipHostMalloc(&c->h_stage, MRG_STAGE_BYTES, hipHostMallocDefault));
        HIPCHK(hipMalloc(&c->d_stage, MRG_STAGE_BYTES));
        for (auto &e : c->ev) HIPCHK(hipEventCreate(&e));
        if (const char *v = getenv("MRG_LDS_CAP")) c->lds_cap = atoi(v);
        *out = c;
    });
}

int mrg_close(mrg_ctx *c) {
    return guard([&] {
        if (!c) return;
        (void)hipSetDevice(c->device);
        (void)hipStreamSynchronize(c->stream);
        for (auto &e : c->ev) (void)hipEventDestroy(e);
        (void)hipFree(c->d_cnt);
        (void)hipHostFree(c->h_cnt);
        if (c->h_stage) (void)hipHostFree(c->h_stage);
        if (c->d_stage) (void)hipFree(c->d_stage);
        if (c->own) (void)hipStreamDestroy(c->own);
        delete c;
    });
}

int mrg_set_stream(mrg_ctx *c, void *hip_stream) {
    return guard([&] {
        if (!c) raise(MRG_EINVAL, "null context");
        sync(c);
        c->stream = hip_stream ? (hipStream_t)hip_stream : c->own;
    });
}

int mrg_set_timing(mrg_ctx *c, int enable) {
    return guard([&] {
        if (!c) raise(MRG_EINVAL, "null context");
        c->timing = enable != 0;
    });
}

int mrg_get_stats(mrg_ctx *c, mrg_stats *out) {
    return guard([&] {
        if (!c || !out) raise(MRG_EINVAL, "null argument");
        *out = c->st;
    });
}

int mrg_job_begin(mrg_ctx *c, int app, uint32_t n_reduce, uint32_t flags) {
    return guard([&] {
        if (!c) raise(MRG_EINVAL, "null context");
        HIPCHK(hipSetDevice(c->device));
        job_begin(c, app, n_reduce, flags);
    });
}

int mrg_job_set_doc_names(mrg_ctx *c, const char *const *names, uint32_t n_names) {
    return guard([&] {
        need_job(c);
        check_names(names, n_names);
        c->names.assign(names, names + n_names);
    });
}

int mrg_job_set_input(mrg_ctx *c, const uint8_t *d_bytes, const uint64_t *h_doc_off, uint32_t n_docs,
                      const uint32_t *h_doc_ids) {
    return guard([&] {
        need_job(c);
        if (!h_doc_off) raise(MRG_EINVAL, "null document offsets (h_doc_off needs n_docs + 1 entries)");
        if (n_docs && !d_bytes) raise(MRG_EINVAL, "null input");
        if (n_docs == 0xFFFFFFFFu) raise(MRG_EINVAL, "n_docs out of range");
        if ((uintptr_t)d_bytes & 15u) raise(MRG_EINVAL, "input buffer must be 16-byte aligned");
        for (uint32_t i = 0; i < n_docs; ++i)
            if (h_doc_off[i + 1] < h_doc_off[i]) raise(MRG_EINVAL, "document offsets must be non-decreasing");
        c->d_in = d_bytes;
        c->doc_off.assign(h_doc_off, h_doc_off + n_docs + 1);
        if (h_doc_ids) c->doc_ids.assign(h_doc_ids, h_doc_ids + n_docs);
        else c->doc_ids.clear();
        c->mapped = c->reduced = false;
    });
}

int mrg_job_map(mrg_ctx *c) {
    return guard([&] { job_map(c); });
}

int mrg_job_export_sizes(mrg_ctx *c, uint32_t n_owners, uint64_t *h_rec_counts, uint64_t *h_heap_bytes) {
    return guard([&] { export_sizes(c, n_owners, h_rec_counts, h_heap_bytes); });
}

int mrg_job_export(mrg_ctx *c, void *d_rec, void *d_heap) {
    return guard([&] { export_pack(c, d_rec, d_heap); });
}

int mrg_job_import(mrg_ctx *c, const void *d_rec, uint64_t n_rec, const void *d_heap, uint64_t heap_bytes,
                   const uint64_t *h_seg_recs, const uint64_t *h_seg_heap, uint32_t n_segs) {
    return guard([&] { job_import(c, d_rec, n_rec, d_heap, heap_bytes, h_seg_recs, h_seg_heap, n_segs); });
}

int mrg_job_reduce(mrg_ctx *c, uint64_t *h_out_bytes) {
    return guard([&] {
        job_reduce(c);
        if (h_out_bytes) *h_out_bytes = c->out_bytes;
    });
}

int mrg_job_output(mrg_ctx *c, const uint8_t **d_out, uint64_t *h_part_off) {
    return guard([&] {
        need_job(c);
        if (!c->reduced) raise(MRG_EINVAL, "no output: call mrg_job_reduce first");
        if (d_out) *d_out = c->d_out;
        if (h_part_off) memcpy(h_part_off, c->part_off.data(), 8ull * (c->R + 1));
    });
}

int mrg_job_copy_output(mrg_ctx *c, uint8_t *h_dst, uint64_t cap) {
    return guard([&] {
        need_job(c);
        if (!c->reduced) raise(MRG_EINVAL, "no output: call mrg_job_reduce first");
        if (cap < c->out_bytes) raise(MRG_EINVAL, "destination too small (%llu < %llu)", (unsigned long long)cap,
                                      (unsigned long long)c->out_bytes);
        if (c->out_bytes)
            HIPCHK(hipMemcpyAsync(h_dst, c->d_out, c->out_bytes, hipMemcpyDeviceToHost, c->stream));
        sync(c);
    });
}

int mrg_job_final(mrg_ctx *c, const uint8_t **d_out, uint64_t *h_bytes) {
    return guard([&] {
        job_final(c);
        if (d_out) *d_out = c->d_final;
        if (h_bytes) *h_bytes = c->final_bytes;
    });
}

int mrg_job_copy_final(mrg_ctx *c, uint8_t *h_dst, uint64_t cap) {
    return guard([&] {
        need_job(c);
        if (!c->finalized) raise(MRG_EINVAL, "no final.txt: call mrg_job_final first");
        if (cap < c->final_bytes) raise(MRG_EINVAL, "destination too small (%llu < %llu)", (unsigned long long)cap,
                                        (unsigned long long)c->final_bytes);
        if (c->final_bytes)
            HIPCHK(hipMemcpyAsync(h_dst, c->d_final, c->final_bytes, hipMemcpyDeviceToHost, c->stream));
        sync(c);
    });
}

// ---- text intermediates
int mrg_map_text(mrg_ctx *c, const uint8_t *h_bytes, size_t n, uint32_t n_reduce, uint8_t **h_out,
                 uint64_t *h_part_off) {
    return guard([&] {
        if (!c || !h_out || !h_part_off || (n && !h_bytes)) raise(MRG_EINVAL, "null argument");
        if (n_reduce == 0) raise(MRG_EINVAL, "n_reduce must be > 0");
        HIPCHK(hipSetDevice(c->device));
        std::vector<uint8_t> out;
        std::vector<uint64_t> off;
        text_map(c, h_bytes, n, n_reduce, out, off);
        uint8_t *o = (uint8_t *)malloc(out.size() + 1);
        if (!o) raise(MRG_ENOMEM, "host allocation failed");
        if (!out.empty()) memcpy(o, out.data(), out.size());
        memcpy(h_part_off, off.data(), 8ull * (n_reduce + 1));
        *h_out = o;
    });
}

int mrg_reduce_text(mrg_ctx *c, const uint8_t *const *h_files, const uint64_t *h_sizes, size_t k, uint32_t flags,
                    uint8_t **h_out, size_t *h_out_len) {
    return guard([&] {
        if (!c || !h_out || !h_out_len || (k && (!h_files || !h_sizes))) raise(MRG_EINVAL, "null argument");
        for (size_t i = 0; i < k; ++i)
            if (h_sizes[i] && !h_files[i]) raise(MRG_EINVAL, "null file %zu", i);
        HIPCHK(hipSetDevice(c->device));
        std::vector<uint8_t> out;
        text_reduce(c, h_files, h_sizes, k, flags, out);
        uint8_t *o = (uint8_t *)malloc(out.size() + 1);
        if (!o) raise(MRG_ENOMEM, "host allocation failed");
        if (!out.empty()) memcpy(o, out.data(), out.size());
        *h_out = o;
        *h_out_len = out.size();
    });
}

// ---- plugin surface (host buffers)

int mrg_map(mrg_ctx *c, int app, const uint8_t *h_bytes, size_t n, const char *doc, uint32_t doc_id,
            uint32_t n_reduce, uint32_t flags, mrg_parts **out) {
    return guard([&] {
        if (!c || !out || (n && !h_bytes)) raise(MRG_EINVAL, "null argument");
        (void)doc;
        HIPCHK(hipSetDevice(c->device));
        job_begin(c, app, n_reduce, flags);
        uint8_t *d = pget<uint8_t>(c->pool, n + 64);
        if (n) HIPCHK(hipMemcpyAsync(d, h_bytes, n, hipMemcpyHostToDevice, c->stream));
        const uint64_t off[2] = {0, n};
        c->d_in = d;
        c->doc_off.assign(off, off + 2);
        c->doc_ids.assign(1, doc_id);
        try {
            job_map(c);
        } catch (...) {
            c->pool.put(d);
            throw;
        }
        export_sizes(c, n_reduce, nullptr, nullptr);
        mrg_parts *P = new mrg_parts();
        P->R = n_reduce;
        P->rec_off.assign(n_reduce + 1, 0);
        P->heap_off.assign(n_reduce + 1, 0);
        for (uint32_t r = 0; r < n_reduce; ++r) {
            P->rec_off[r + 1] = P->rec_off[r] + c->exp_rec[r];
            P->heap_off[r + 1] = P->heap_off[r] + c->exp_heap[r];
        }
        XRec *dx = pget<XRec>(c->pool, P->rec_off[n_reduce]);
        uint8_t *dh = pget<uint8_t>(c->pool, P->heap_off[n_reduce] + 1);
        export_pack(c, dx, dh);
        P->recs.resize(P->rec_off[n_reduce] * sizeof(XRec));
        P->heap.resize(P->heap_off[n_reduce]);
        if (!P->recs.empty())
            HIPCHK(hipMemcpyAsync(P->recs.data(), dx, P->recs.size(), hipMemcpyDeviceToHost, c->stream));
        if (!P->heap.empty())
            HIPCHK(hipMemcpyAsync(P->heap.data(), dh, P->heap.size(), hipMemcpyDeviceToHost, c->stream));
        sync(c);
        c->pool.put(dx);
        c->pool.put(dh);
        c->pool.put(d);
        *out = P;
    });
}

int mrg_parts_get(const mrg_parts *P, uint32_t r, const uint8_t **h_rec, uint64_t *n_rec, const uint8_t **h_heap,
                  uint64_t *heap_bytes) {
    return guard([&] {
        if (!P || r >= P->R) raise(MRG_EINVAL, "bad parts / partition");
        if (h_rec) *h_rec = P->recs.data() + P->rec_off[r] * sizeof(XRec);
        if (n_rec) *n_rec = P->rec_off[r + 1] - P->rec_off[r];
        if (h_heap) *h_heap = P->heap.data() + P->heap_off[r];
        if (heap_bytes) *heap_bytes = P->heap_off[r + 1] - P->heap_off[r];
    });
}

void mrg_parts_free(mrg_parts *P) { delete P; }

int mrg_reduce(mrg_ctx *c, int app, uint32_t r, const mrg_parts *const *in, size_t k, uint32_t n_reduce,
               uint32_t flags, const char *const *doc_names, uint32_t n_docs, uint8_t **h_out, size_t *h_out_len) {
    return guard([&] {
        if (!c || !h_out || !h_out_len || (k && !in)) raise(MRG_EINVAL, "null argument");
        if (r >= n_reduce) raise(MRG_EINVAL, "partition %u >= n_reduce %u", r, n_reduce);
        HIPCHK(hipSetDevice(c->device));
        job_begin(c, app, n_reduce, flags);
        if (app == MRG_APP_INDEXER) {
            check_names(doc_names, n_docs);
            c->names.assign(doc_names, doc_names + n_docs);
        }
        std::vector<uint64_t> seg_rec, seg_heap;
        std::vector<uint8_t> recs, heap;
        for (size_t i = 0; i < k; ++i) {
            const mrg_parts *P = in[i];
            if (!P || P->R != n_reduce) raise(MRG_EINVAL, "map output %zu has a different n_reduce", i);
            const uint64_t a = P->rec_off[r], b = P->rec_off[r + 1];
            const uint64_t ha = P->heap_off[r], hb = P->heap_off[r + 1];
            recs.insert(recs.end(), P->recs.begin() + a * sizeof(XRec), P->recs.begin() + b * sizeof(XRec));
            heap.insert(heap.end(), P->heap.begin() + ha, P->heap.begin() + hb);
            seg_rec.push_back(b - a);
            seg_heap.push_back(hb - ha);
        }
        const uint64_t nrec = recs.size() / sizeof(XRec);
        uint8_t *dr = pget<uint8_t>(c->pool, recs.size() + 16);
        uint8_t *dh = pget<uint8_t>(c->pool, heap.size() + 16);
        if (!recs.empty()) HIPCHK(hipMemcpyAsync(dr, recs.data(), recs.size(), hipMemcpyHostToDevice, c->stream));
        if (!heap.empty()) HIPCHK(hipMemcpyAsync(dh, heap.data(), heap.size(), hipMemcpyHostToDevice, c->stream));
        job_import(c, dr, nrec, dh, heap.size(), seg_rec.data(), seg_heap.data(), (uint32_t)seg_rec.size());
        job_reduce(c);
        const uint64_t a = c->part_off[r], b = c->part_off[r + 1];
        uint8_t *o = (uint8_t *)malloc(b - a + 1);
        if (!o) raise(MRG_ENOMEM, "host allocation failed");
        if (b > a) HIPCHK(hipMemcpyAsync(o, c->d_out + a, b - a, hipMemcpyDeviceToHost, c->stream));
        sync(c);
        c->pool.put(dr);
        c->pool.put(dh);
        *h_out = o;
        *h_out_len = b - a;
    });
}

int mrg_comm_get_id(uint8_t id[MRG_COMM_ID_BYTES]) {
    return guard([&] {
        if (!id) raise(MRG_EINVAL, "null id");
        static_assert(sizeof(ncclUniqueId) == MRG_COMM_ID_BYTES, "RCCL unique id size");
        ncclUniqueId u;
        NCCLCHK(ncclGetUniqueId(&u));
        memcpy(id, &u, sizeof u);
    });
}

int mrg_comm_init(mrg_ctx *c, const uint8_t id[MRG_COMM_ID_BYTES], int n_ranks, int rank, mrg_comm **out) {
    return guard([&] {
        if (!c || !id || !out) raise(MRG_EINVAL, "null argument");
        if (n_ranks < 1 || rank < 0 || rank >= n_ranks) raise(MRG_EINVAL, "rank %d of %d", rank, n_ranks);
        HIPCHK(hipSetDevice(c->device));
        ncclUniqueId u;
        memcpy(&u, id, sizeof u);
        // the buffers first: a rank that fails here has not joined, and its peers' init fails or
        // waits for it (the caller's concern: mrg_run_job creates its communicators in one call)
        mrg_comm *m = comm_alloc(c->device, n_ranks, rank);
        const ncclResult_t r = ncclCommInitRank(&m->comm, n_ranks, u, rank);
        if (r != ncclSuccess) {
            comm_free(m);
            raise(MRG_ECOMM, "ncclCommInitRank(%d of %d): %s", rank, n_ranks, ncclGetErrorString(r));
        }
        *out = m;
    });
}

int mrg_comm_destroy(mrg_comm *m) {
    return guard([&] {
        if (!m) return;
        ncclResult_t r = ncclSuccess;
        if (m->comm && !m->aborted.load()) {
            (void)hipSetDevice(m->device);
            r = ncclCommDestroy(m->comm);
        }
        m->comm = nullptr;
        comm_free(m);
        if (r != ncclSuccess) raise(MRG_ECOMM, "ncclCommDestroy: %s", ncclGetErrorString(r));
    });
}

int mrg_job_shuffle(mrg_ctx *c, mrg_comm *m) {
    return guard([&] { job_shuffle(c, m); });
}

int mrg_comm_count(const mrg_comm *m, int *n_ranks) {
    return guard([&] {
        if (!m || !n_ranks) raise(MRG_EINVAL, "null argument");
        if (!m->comm || m->aborted.load()) raise(MRG_ECOMM, "the communicator was aborted");
        int n = 0;
        const ncclResult_t r = ncclCommCount(m->comm, &n);
        if (r != ncclSuccess) raise(MRG_ECOMM, "ncclCommCount: %s", ncclGetErrorString(r));
        *n_ranks = n;
    });
}

int mrg_pool_stats(mrg_ctx *c, uint64_t *outstanding, uint64_t *held_bytes) {
    return guard([&] {
        if (!c) raise(MRG_EINVAL, "null context");
        if (outstanding) *outstanding = c->pool.outstanding();
        if (held_bytes) *held_bytes = c->pool.held_bytes();
    });
}

int mrg_pool_alloc_stats(mrg_ctx *c, uint64_t *n_allocs, uint64_t *alloc_bytes, double *alloc_ms) {
    return guard([&] {
        if (!c) raise(MRG_EINVAL, "null context");
        c->pool.alloc_stats(n_allocs, alloc_bytes, alloc_ms);
    });
}

}  // extern "C"

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

thread_local mrg_run_stats g_run{};

void write_file(const std::string &path, const uint8_t *p, uint64_t n) {
    FILE *f = fopen(path.c_str(), "wb");  // worker.rs:167-168 File::create("mr-{r}.txt")
    if (!f) raise(MRG_EIO, "cannot create %s", path.c_str());
    const size_t w = n ? fwrite(p, 1, n, f) : 0;
    const int cl = fclose(f);
    if (w != n || cl != 0) raise(MRG_EIO, "short write on %s", path.c_str());
}

// k-way merge of G byte-sorted line runs (each GPU's final.txt lines): LC_ALL=C `sort` order.  A run
// may lack its final newline (its last line then ends at the run's end); each cursor's line end is
// found once per line.
std::vector<uint8_t> merge_sorted_lines(const std::vector<std::pair<const uint8_t *, uint64_t>> &runs) {
    struct Cur { const uint8_t *p, *e, *le; };  // le = end of the current line (its '\n' or e)
    std::vector<Cur> cur;
    uint64_t total = 0;
    auto line_end = [](const uint8_t *p, const uint8_t *e) {
        const uint8_t *q = (const uint8_t *)memchr(p, '\n', (size_t)(e - p));
        return q ? q : e;
    };
    for (auto &r : runs) {
        if (!r.second) continue;
        cur.push_back({r.first, r.first + r.second, line_end(r.first, r.first + r.second)});
        total += r.second;
    }
    std::vector<uint8_t> out;
    out.reserve(total + runs.size());
    while (!cur.empty()) {
        size_t best = 0;
        for (size_t i = 1; i < cur.size(); ++i) {
            const size_t la = (size_t)(cur[i].le - cur[i].p), lb = (size_t)(cur[best].le - cur[best].p);
            const int cm = memcmp(cur[i].p, cur[best].p, std::min(la, lb));
            if (cm < 0 || (cm == 0 && la < lb)) best = i;
        }
        Cur &c = cur[best];
        out.insert(out.end(), c.p, c.le);
        out.push_back('\n');  // every output line ends with a newline, also a run's unterminated last one
        c.p = c.le < c.e ? c.le + 1 : c.e;
        if (c.p >= c.e) cur.erase(cur.begin() + (ptrdiff_t)best);
        else c.le = line_end(c.p, c.e);
    }
    return out;
}

// ---- input files -> device: worker.rs:65-77 reads each file whole (read_to_string).  Here the
// files of a GPU are read in chunks by several host threads into pinned staging buffers (two per
// thread), each chunk copied to the device buffer while the thread reads the next one, so disk /
// page-cache reads and the PCIe copies overlap.
struct FileChunk {
    uint32_t file;   // index in the rank's file list
    uint64_t off, n; // bytes [off, off + n) of the file
    uint64_t dst;    // offset in the device buffer
};

constexpr uint64_t MRG_READ_CHUNK = 32ull << 20;

void read_files_to_device(int device, const std::vector<const char *> &paths, const std::vector<uint64_t> &doc_off,
                          uint8_t *d, int n_threads) {
    std::vector<FileChunk> chunks;
    for (uint32_t i = 0; i < paths.size(); ++i) {
        const uint64_t sz = doc_off[i + 1] - doc_off[i];
        for (uint64_t o = 0; o < sz; o += MRG_READ_CHUNK)
            chunks.push_back({i, o, std::min<uint64_t>(MRG_READ_CHUNK, sz - o), doc_off[i] + o});
    }
    if (chunks.empty()) return;
    n_threads = std::max(1, std::min<int>(n_threads, (int)chunks.size()));
    uint64_t pin_bytes = 0;  // staging buffers sized to the largest chunk (small inputs: small buffers)
    for (auto &ch : chunks) pin_bytes = std::max(pin_bytes, ch.n);
    std::atomic<size_t> next{0};
    std::atomic<int> fail{0};
    std::vector<int> rc(n_threads, MRG_OK);
    std::vector<std::string> msg(n_threads);
    auto reader = [&](int t) {
        rc[t] = guard([&] {
            HIPCHK(hipSetDevice(device));
            hipStream_t st = nullptr;
            uint8_t *pin[2] = {nullptr, nullptr};
            hipEvent_t ev[2] = {nullptr, nullptr};
            std::vector<int> fds(paths.size(), -1);
            struct Res {  // released on every exit path
                hipStream_t &st; uint8_t **pin; hipEvent_t *ev; std::vector<int> &fds;
                ~Res() {
                    if (st) (void)hipStreamSynchronize(st);
                    for (int k = 0; k < 2; ++k) { if (ev[k]) (void)hipEventDestroy(ev[k]); if (pin[k]) (void)hipHostFree(pin[k]); }
                    if (st) (void)hipStreamDestroy(st);
                    for (int fd : fds) if (fd >= 0) close(fd);
                }
            } res{st, pin, ev, fds};
            HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            for (int k = 0; k < 2; ++k) {
                HIPCHK(hipHostMalloc(&pin[k], pin_bytes, hipHostMallocDefault));
                HIPCHK(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming));
            }
            bool used[2] = {false, false};
            for (int k = 0;; k ^= 1) {
                if (fail.load()) return;
                const size_t ci = next.fetch_add(1);
                if (ci >= chunks.size()) break;
                const FileChunk &ch = chunks[ci];
                if (used[k]) HIPCHK(hipEventSynchronize(ev[k]));  // the copy out of this buffer is done
                int &fd = fds[ch.file];
                if (fd < 0) {
                    fd = open(paths[ch.file], O_RDONLY);  // worker.rs:73 File::open(..).unwrap()
                    if (fd < 0) raise(MRG_EIO, "cannot open %s", paths[ch.file]);
                }
                uint64_t got = 0;
                while (got < ch.n) {
                    const ssize_t r = pread(fd, pin[k] + got, (size_t)(ch.n - got), (off_t)(ch.off + got));
                    if (r <= 0) raise(MRG_EIO, "short read on %s", paths[ch.file]);
                    got += (uint64_t)r;
                }
                HIPCHK(hipMemcpyAsync(d + ch.dst, pin[k], ch.n, hipMemcpyHostToDevice, st));
                HIPCHK(hipEventRecord(ev[k], st));
                used[k] = true;
            }
            HIPCHK(hipStreamSynchronize(st));
        });
        if (rc[t]) {
            msg[t] = g_err;
            fail.store(1);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < n_threads; ++t) th.emplace_back(reader, t);
    reader(0);
    for (auto &x : th) x.join();
    for (int t = 0; t < n_threads; ++t)
        if (rc[t]) raise(rc[t], "%s", msg[t].c_str());
}

// One GPU of mrg_run_job.
struct RankState {
    int g = 0, device = 0;
    mrg_ctx *c = nullptr;
    mrg_comm *m = nullptr;
    uint8_t *d = nullptr;
    uint64_t in_bytes = 0;
    std::vector<uint8_t> out, fin;
};

// Runs fn on every rank, one host thread each, and returns when all have returned; the per-rank
// status codes and messages are left in rc / msg.  In a phase with collectives (`watch`), a rank
// that failed outside the exchange's own status protocol (an RCCL error) can leave its peers
// waiting for it: once a rank has failed and the others have not finished within the grace period
// (MRG_ABORT_GRACE_MS, default 10 s), every communicator is aborted, so the waiting RCCL operations
// fail and their threads return.
template <class F>
void run_ranks(std::vector<RankState> &rs, bool watch, F &&fn, std::vector<int> &rc, std::vector<std::string> &msg) {
    const int G = (int)rs.size();
    rc.assign(G, MRG_OK);
    msg.assign(G, std::string());
    std::mutex mu;
    std::condition_variable cv;
    int done = 0, failed = 0;
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g)
        th.emplace_back([&, g] {
            const int r = guard([&] {
                HIPCHK(hipSetDevice(rs[g].device));
                fn(rs[g]);
            });
            std::lock_guard<std::mutex> lk(mu);
            rc[g] = r;
            if (r) {
                msg[g] = g_err;
                ++failed;
            }
            ++done;
            cv.notify_all();
        });
    const uint64_t grace_ms = env_u64("MRG_ABORT_GRACE_MS", 10000);
    {
        std::unique_lock<std::mutex> lk(mu);
        Clock::time_point first_fail{};
        bool aborted = false;
        while (done < G) {
            cv.wait_for(lk, std::chrono::milliseconds(50));
            if (!watch || aborted || !failed || done >= G) continue;
            if (first_fail == Clock::time_point{}) first_fail = Clock::now();
            if (ms_since(first_fail) < (double)grace_ms) continue;
            aborted = true;
            lk.unlock();  // the rank threads report in while their communicators are aborted
            const auto deadline = Clock::now() + std::chrono::milliseconds(2000);
            std::vector<std::thread> ab;
            for (auto &r : rs)
                if (r.m) ab.emplace_back([m = r.m, deadline] { comm_abort(m, deadline); });
            for (auto &t : ab) t.join();
            lk.lock();
        }
    }
    for (auto &t : th) t.join();
}

// The first failure that is not an echo (MRG_ECOMM) of another rank's, else the first failure.
void raise_first(const std::vector<int> &rc, const std::vector<std::string> &msg, const std::vector<RankState> &rs) {
    for (size_t g = 0; g < rc.size(); ++g)
        if (rc[g] && rc[g] != MRG_ECOMM) raise(rc[g], "GPU %d: %s", rs[g].device, msg[g].c_str());
    for (size_t g = 0; g < rc.size(); ++g)
        if (rc[g]) raise(rc[g], "GPU %d: %s", rs[g].device, msg[g].c_str());
}

void release_ranks(std::vector<RankState> &rs) {
    for (auto &r : rs) {
        if (r.d && r.c) {
            (void)hipSetDevice(r.device);
            r.c->pool.put(r.d);
        }
        if (r.m) (void)mrg_comm_destroy(r.m);
        if (r.c) (void)mrg_close(r.c);
        r = RankState{};
    }
}

// The whole job on GPUs devices[0..G): the static plan for the coordinator's task assignment
// (coordinator.rs:137-215) and the workers' map-then-reduce loop (mrworker.rs:43-149).  Phases, each
// on all GPUs at once and joined before the next: open contexts -> create the communicators (one
// ncclCommInitAll) -> read + map -> exchange -> reduce + write.  A failure in any phase fails the job
// there: before the communicators exist nothing collective has started, and the exchange agrees on
// every rank's status before each of its transfers, so no GPU thread is left waiting for another.
void run_job(const char *const *files, size_t n_files, uint32_t R, int app, const char *out_dir, uint32_t flags,
             const std::vector<int> &devices) {
    const Clock::time_point t_all = Clock::now();
    g_run = mrg_run_stats{};
    const int G = (int)devices.size();
    g_run.n_gpus = G;
    std::vector<const char *> names(files, files + n_files);
    check_names(names.data(), (uint32_t)n_files);
    std::vector<RankState> rs(G);
    struct Guard { std::vector<RankState> &rs; ~Guard() { release_ranks(rs); } } release{rs};
    std::vector<int> rc;
    std::vector<std::string> msg;
    // ---- contexts (worker processes)
    Clock::time_point t0 = Clock::now();
    for (int g = 0; g < G; ++g) {
        rs[g].g = g;
        rs[g].device = devices[g];
        test_fail("open", g);
        if (mrg_open(devices[g], &rs[g].c) != MRG_OK) raise(MRG_EHIP, "GPU %d: %s", devices[g], mrg_last_error());
    }
    // ---- communicators: all of them in one call (nothing to wait for if one cannot be made)
    const bool comm = G > 1 || env_u64("MRG_TEST_FORCE_COMM", 0);
    if (comm) {
        test_fail("comm", 0);
        std::vector<ncclComm_t> cs(G, nullptr);
        const ncclResult_t r = ncclCommInitAll(cs.data(), G, devices.data());
        if (r != ncclSuccess) raise(MRG_ECOMM, "ncclCommInitAll over %d GPUs: %s", G, ncclGetErrorString(r));
        for (int g = 0; g < G; ++g) {
            try {
                rs[g].m = comm_alloc(devices[g], G, g);
            } catch (...) {
                for (int k = g; k < G; ++k) { (void)hipSetDevice(devices[k]); (void)ncclCommDestroy(cs[k]); }
                throw;
            }
            rs[g].m->comm = cs[g];
        }
    }
    g_run.ms_open = ms_since(t0);
    // ---- map phase: GPU g reads and maps files m with m % G == g (coordinator.rs:137-176)
    const int readers = (int)std::max<uint64_t>(1, env_u64("MRG_READ_THREADS", std::max(1, std::min(16, 32 / G))));
    std::vector<double> t_read(G, 0.0), t_alloc(G, 0.0), t_mapk(G, 0.0), t_aggk(G, 0.0);
    t0 = Clock::now();
    run_ranks(rs, false, [&](RankState &r) {
        mrg_ctx *c = r.c;
        test_fail("map", r.g);
        const Clock::time_point tr = Clock::now();
        job_begin(c, app, R, flags);
        c->names.assign(files, files + n_files);
        std::vector<const char *> mine;
        std::vector<uint64_t> off(1, 0);
        std::vector<uint32_t> ids;
        for (size_t m = (size_t)r.g; m < n_files; m += (size_t)G) {
            struct stat sb;
            if (stat(files[m], &sb) != 0) raise(MRG_EIO, "cannot open %s", files[m]);  // worker.rs:73
            mine.push_back(files[m]);
            off.push_back(off.back() + (uint64_t)sb.st_size);
            ids.push_back((uint32_t)m);
        }
        r.in_bytes = off.back();
        r.d = pget<uint8_t>(c->pool, off.back() + 64);
        read_files_to_device(c->device, mine, off, r.d, readers);
        t_read[r.g] = ms_since(tr);
        c->d_in = r.d;
        c->doc_off = off;
        c->doc_ids = ids;
        double a0 = 0.0, a1 = 0.0;
        c->pool.alloc_stats(nullptr, nullptr, &a0);
        c->timing = true;  // HIP events around the map and aggregation kernels (mrg_run_stats)
        job_map(c);
        c->pool.alloc_stats(nullptr, nullptr, &a1);
        t_alloc[r.g] = a1 - a0;
        t_mapk[r.g] = c->st.ms_map;
        t_aggk[r.g] = c->st.ms_aggregate;
    }, rc, msg);
    raise_first(rc, msg, rs);
    g_run.ms_map = ms_since(t0);
    for (int g = 0; g < G; ++g) {
        g_run.ms_map_alloc = std::max(g_run.ms_map_alloc, t_alloc[g]);
        g_run.ms_map_kernel = std::max(g_run.ms_map_kernel, t_mapk[g]);
        g_run.ms_aggregate_kernel = std::max(g_run.ms_aggregate_kernel, t_aggk[g]);
        g_run.ms_read = std::max(g_run.ms_read, t_read[g]);
        g_run.input_bytes += rs[g].in_bytes;
    }
    g_run.ms_map -= g_run.ms_read;
    // ---- exchange (RCCL over xGMI)
    if (comm) {
        t0 = Clock::now();
        run_ranks(rs, true, [&](RankState &r) { job_shuffle(r.c, r.m); }, rc, msg);
        raise_first(rc, msg, rs);
        g_run.ms_shuffle = ms_since(t0);
    }
    // ---- reduce phase: GPU g formats the partitions r % G == g (coordinator.rs:178-215)
    t0 = Clock::now();
    run_ranks(rs, false, [&](RankState &r) {
        mrg_ctx *c = r.c;
        test_fail("reduce", r.g);
        job_reduce(c);
        r.out.resize(c->out_bytes);
        if (c->out_bytes) HIPCHK(hipMemcpyAsync(r.out.data(), c->d_out, c->out_bytes, hipMemcpyDeviceToHost, c->stream));
        if (flags & MRG_FLAG_FINAL_TXT) {  // run.sh:16-20 generate_output: this GPU's lines, sorted on the device
            job_final(c);
            r.fin.resize(c->final_bytes);
            if (c->final_bytes)
                HIPCHK(hipMemcpyAsync(r.fin.data(), c->d_final, c->final_bytes, hipMemcpyDeviceToHost, c->stream));
        }
        sync(c);
    }, rc, msg);
    raise_first(rc, msg, rs);
    g_run.ms_reduce = ms_since(t0);
    // ---- writes: mr-{r}.txt by the GPU that owns r (worker.rs:167-179), then final.txt
    t0 = Clock::now();
    run_ranks(rs, false, [&](RankState &r) {
        test_fail("write", r.g);
        for (uint32_t p = (uint32_t)r.g; p < R; p += (uint32_t)G) {
            const uint64_t a = r.c->part_off[p], b = r.c->part_off[p + 1];
            write_file(std::string(out_dir) + "/mr-" + std::to_string(p) + ".txt", r.out.data() + a, b - a);
        }
    }, rc, msg);
    raise_first(rc, msg, rs);
    for (auto &r : rs) g_run.output_bytes += r.out.size();
    if (flags & MRG_FLAG_FINAL_TXT) {
        std::vector<std::pair<const uint8_t *, uint64_t>> runs;
        for (auto &r : rs) runs.push_back({r.fin.data(), r.fin.size()});
        if (G == 1) write_file(std::string(out_dir) + "/final.txt", rs[0].fin.data(), rs[0].fin.size());
        else {
            const std::vector<uint8_t> all = merge_sorted_lines(runs);
            write_file(std::string(out_dir) + "/final.txt", all.data(), all.size());
        }
    }
    g_run.ms_write = ms_since(t0);
    g_run.ms_total = ms_since(t_all);
}

}  // namespace

extern "C" {

int mrg_run_job(const char *const *files, size_t n_files, uint32_t n_reduce, int app, const char *out_dir,
                uint32_t flags, int n_gpus) {
    return guard([&] {
        if ((n_files && !files) || !out_dir) raise(MRG_EINVAL, "null argument");
        if (n_reduce == 0) raise(MRG_EINVAL, "n_reduce must be > 0");
        int ndev = 0;
        HIPCHK(hipGetDeviceCount(&ndev));
        if (n_gpus < 1 || n_gpus > ndev) raise(MRG_EINVAL, "n_gpus %d: %d devices visible", n_gpus, ndev);
        std::vector<int> devs(n_gpus);
        for (int g = 0; g < n_gpus; ++g) devs[g] = g;
        run_job(files, n_files, n_reduce, app, out_dir, flags, devs);
    });
}

int mrg_run_get_stats(mrg_run_stats *out) {
    return guard([&] {
        if (!out) raise(MRG_EINVAL, "null argument");
        *out = g_run;
    });
}

// Test entry (not in include/mrgpu.h): the k-way merge of sorted line runs that builds a multi-GPU
// final.txt, callable without a GPU.  *out (free with mrg_free) receives the merged bytes.
int mrg_test_merge_sorted_lines(const uint8_t *const *runs, const uint64_t *sizes, size_t k, uint8_t **out,
                                uint64_t *out_len) {
    return guard([&] {
        if (!out || !out_len || (k && (!runs || !sizes))) raise(MRG_EINVAL, "null argument");
        std::vector<std::pair<const uint8_t *, uint64_t>> v;
        for (size_t i = 0; i < k; ++i) v.push_back({runs[i], sizes[i]});
        const std::vector<uint8_t> m = merge_sorted_lines(v);
        uint8_t *o = (uint8_t *)malloc(m.size() + 1);
        if (!o) raise(MRG_ENOMEM, "host allocation failed");
        if (!m.empty()) memcpy(o, m.data(), m.size());
        *out = o;
        *out_len = m.size();
    });
}

void mrg_free(void *p) { free(p); }

int mrg_gen_zipf(mrg_ctx *c, uint8_t *d_dst, uint64_t n_bytes, uint64_t seed, uint64_t file_index, uint32_t vocab,
                 double s) {
    return guard([&] {
        if (!c || (n_bytes && !d_dst)) raise(MRG_EINVAL, "null argument");
        HIPCHK(hipSetDevice(c->device));
        if (mrg_gen_zipf_impl(d_dst, n_bytes, seed, file_index, vocab, s, 0, c->stream))
            raise(MRG_EHIP, "zipf generator failed: %s", hipGetErrorString(hipGetLastError()));
    });
}

int mrg_gen_text(mrg_ctx *c, uint8_t *d_dst, uint64_t n_bytes, uint64_t seed, uint64_t file_index, uint32_t vocab,
                 double s, uint32_t style) {
    return guard([&] {
        if (!c || (n_bytes && !d_dst)) raise(MRG_EINVAL, "null argument");
        if (style > MRG_TEXT_GUTENBERG) raise(MRG_EINVAL, "unknown text style %u", style);
        HIPCHK(hipSetDevice(c->device));
        if (mrg_gen_zipf_impl(d_dst, n_bytes, seed, file_index, vocab, s, style, c->stream))
            raise(MRG_EHIP, "text generator failed: %s", hipGetErrorString(hipGetLastError()));
    });
}

int mrg_gen_unique(mrg_ctx *c, uint8_t *d_dst, uint64_t n_bytes, uint64_t seed, uint64_t file_index) {
    return guard([&] {
        if (!c || (n_bytes && !d_dst)) raise(MRG_EINVAL, "null argument");
        HIPCHK(hipSetDevice(c->device));
        if (mrg_gen_unique_impl(d_dst, n_bytes, seed, file_index, c->stream))
            raise(MRG_EHIP, "unique generator failed: %s", hipGetErrorString(hipGetLastError()));
    });
}

}  // extern "C"
