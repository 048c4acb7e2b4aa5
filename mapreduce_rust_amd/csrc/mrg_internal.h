// mrg_internal.h -- host-side declarations shared by the kernel files and the C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#ifndef MRG_MAP_WAVES  // (timing variants override it: the r06 occupancy sweep)
#define MRG_MAP_WAVES 16        // waves per map workgroup (one workgroup per CU, one shared LDS table)
#endif
#define MRG_MAP_WG (64 * MRG_MAP_WAVES)
#define MRG_MAP_SEG 16          // input bytes per lane per tile
#define MRG_MAP_TILE (64 * MRG_MAP_SEG)  // 1 KiB tile per WAVE iteration (waves never synchronise)
#define MRG_MAP_HALO 64         // bytes after the tile staged in LDS (tokens crossing the tile end)
#define MRG_MAP_BEHIND 16       // bytes before the tile staged in LDS (previous codepoint)
#define MRG_MAP_NSUB 2          // 1 KiB tiles per wave iteration (one block, prefetched one block ahead)

// Tail records (LDS-table misses) are bucketed by key hash into MRG_NBUCKET buckets; every
// (bucket, map workgroup) pair owns a private region of the pool, so appending is an LDS atomic.
// One workgroup per bucket later sums them in LDS (k_keys.hip).
#ifndef MRG_NBUCKET_LOG2
#define MRG_NBUCKET_LOG2 8  // 256: half the open tail lines of 512 (map 8.1 -> 7.5 ms at C3)
#endif
#define MRG_NBUCKET (1 << MRG_NBUCKET_LOG2)
#define MRG_BA_CAP 7680          // max LDS table slots of the per-bucket aggregation kernel (k_keys.hip ba_cap)
// bytes of one tail record in MapArgs::pool: wc 12 ({k0, high word of k1}: keys of <= 12 bytes, whose
// k1 low word is 0 -- keys never contain NUL), the indexer 24 ({k0, k1, doc}); wc keys of 13..16
// bytes go to the 16-byte pool (MapArgs::pool16)
#define MRG_TAIL_BYTES(idx) ((idx) ? 24u : 12u)

// counters[] slots written by the kernels
enum {
    CNT_REC = 0,      // tail records written by the map kernel
    CNT_LONG = 1,     // long-token records
    CNT_TOKENS = 2,   // tokens
    CNT_ERRPOS = 3,   // first invalid UTF-8 byte (atomicMin), ~0 if none
    CNT_KEYS = 4,     // distinct keys appended to the KeySet
    CNT_OVF = 5,      // tail records that found neither region nor overflow-list room (rerun)
    CNT_OVF2 = 6,     // keys that did not fit their bucket's LDS table (exact overflow path)
    CNT_NONASCII = 7, // 1 KiB tiles that took the non-ASCII tokenizer
    CNT_REC16 = 8,    // of CNT_REC: 16-byte tail records (wc keys of 13..16 bytes)
    CNT_LONGX = 9,    // long-token records beyond their workgroup's region (the shared list)
    CNT_W16 = 10,     // wide map, 12-byte regions: keys of 13..16 bytes that found their bucket's list full
    CNT_N = 11
};

// Stream-ordered caching allocator interface (all work of a context runs on one stream, so a
// buffer released after its last enqueued use can be handed out again immediately).
struct DevPool {
    virtual void *get(size_t bytes) = 0;
    virtual void put(void *p) = 0;
    virtual ~DevPool() {}
};

struct MapArgs {
    const uint8_t *in;
    const uint64_t *doc_off;     // [n_docs + 1] byte offsets into `in`
    const uint64_t *chunk_base;  // [n_docs + 1] first tile index of each document
    const uint32_t *doc_id;      // [n_docs] global document id
    uint32_t n_docs;
    uint64_t n_chunks;
    // tail records (LDS-table misses, count 1): map workgroup w appends the records of bucket b to
    // pool records [rbase[b] + w * bcap[b], + bcap[b]); record i = MRG_TAIL_BYTES(indexer) bytes at
    // (uint8_t *)pool + i * MRG_TAIL_BYTES: wc {u64 k0, u32 high word of k1} for keys of <= 12 bytes,
    // the indexer {k0, k1, doc} (24 B)
    uint64_t *pool;
    const uint64_t *rbase;       // [NBUCKET] first record of bucket b's regions
    const uint32_t *bcap;        // [NBUCKET] records per (bucket, workgroup) region
    uint32_t *bcount;            // [grid * NBUCKET] records appended (may exceed bcap)
    // wc keys of 13..16 bytes: 16-byte records {k0, k1} in their own regions, the same layout
    uint64_t *pool16;
    const uint64_t *rbase16;
    const uint32_t *bcap16;
    uint32_t *bcount16;
    // records beyond their region's capacity: bucket b's overflow list, records
    // [b * ocap, b * ocap + min(onext[b], ocap)) of `ovf` (a full list forces a rerun)
    uint64_t *ovf;
    uint32_t *onext;             // [NBUCKET]
    uint32_t ocap;
    // LDS-table flush: workgroup g writes its entries to [g * CAP, ...) sorted by bucket;
    // foff[g * (NBUCKET + 1) + b] = start of bucket b in that region
    uint64_t *fk0, *fk1;
    uint32_t *fcnt, *fdoc, *foff;
    // long-key token records (> 16 key bytes): map workgroup w appends to its region, records
    // [w * lper, + lper), through an LDS cursor; beyond it to the shared list [grid * lper, + lovf)
    // (a device atomic each; a full list reruns the launch).  lcount[w] = records workgroup w produced
    // (may exceed lper); mrg_launch_long_compact packs them densely afterwards.
    uint64_t *lstart;
    uint32_t *llen, *ldoc;
    uint32_t lper;
    uint64_t lovf;
    uint32_t *lcount;
    // non-ASCII tiles, recorded by the main loop and processed after it: workgroup g appends the
    // index of each such tile (block * NSUB + tile, absolute) to gbits[g * kwords ..)
    uint32_t *gbits;
    uint32_t kwords;             // list capacity per workgroup (tiles of its share + its steal budget)
    unsigned long long *counters;
    uint32_t hash_bits;          // 0 = full; else truncate internal hashes (collision test knob)
    uint32_t ablate;             // perf diagnostics only (env MRG_ABLATE; results are WRONG when set):
                                 // 1 = no tail-record stores, 2 = no LDS-table probe (all tokens
                                 // become tail records), 4 = no per-token work after the queue,
                                 // 8 = every block loads its document's first block (L2-resident),
                                 // 16 = no LDS count add on table hits, 32 = classification
                                 // only, 64 = no queue writes (and no tokens), 128 = every slow
                                 // token through the codepoint walker (results exact: an A/B knob),
                                 // 256 = no UTF-8 class fix of non-ASCII blocks, 512 = no slow
                                 // tokens, 1024 = no squeeze of multi-byte gaps
    unsigned long long *prof;    // perf diagnostics (env MRG_PROF): per-phase wave clocks, [7]; else null
    // wide map (near-unique keys, wc): no LDS combine -- every short key goes
    // straight to its L1 bucket b = partition * wB1r + quantile (SipHash-1-3 % R, then the splitters of a
    // sample of the input), into the region of (b, this workgroup): records
    // [(b * grid + w) * wcap, + wcap) of wrec, 16 bytes {k0, k1} each; wcnt[b * grid + w] = records the
    // workgroup produced for b (may exceed wcap: the launch is then rerun with larger regions)
    uint64_t *wrec;
    uint32_t *wcnt;
    const uint64_t *wspl;        // [wR][wB1r - 1] splitter keys (k0, k1)
    const uint8_t *wix;          // [wR][MRG_WIDE_IX1] splitter index (null: binary search)
    uint32_t wR, wB1r, wcap;
    // w12: the regions hold 12-byte records {k0, high word of k1} (keys of <= 12 bytes; 4 bytes of slack
    // after the last region); a key of 13..16 bytes goes to its bucket's list of 16-byte records,
    // wl16 records [b * wl16cap, + wl16n[b]) (a device atomic each: such keys are rare when w12 is
    // chosen; a full list counts in CNT_W16 and reruns the launch with 16-byte regions)
    uint32_t w12, wl16cap;
    uint64_t *wl16;
    uint32_t *wl16n;
    // load balance (mrgpu.cpp map_steal): blocks [0, n_static) are split into
    // equal workgroup shares; blocks [n_static, n_chunks) are a pool in 8 parts, part j's next block at
    // pool_ctr[16 * j] (zeroed per launch), that a wave takes MRG_MAP_STEAL_K blocks at a time once its
    // workgroup's share is done, at most steal_max blocks per workgroup (the per-workgroup capacities
    // are sized for share + steal_max).  n_static = n_chunks: static shares only.
    uint64_t n_static;
    uint32_t steal_max;
    unsigned long long *pool_ctr;
};
// One staged small write of a job's setup (mrgpu.cpp stage_h2d / stage_fill): `n` bytes to `dst`, from
// offset `src` of the device copy of the pinned staging buffer, or the byte `fill` when src == ~0u.
// A batch of them is one host-to-device copy and one k_stage_scatter launch (was one copy or memset
// each, ~8 us apiece on the stream).
struct StageOp {
    uint64_t dst;
    uint32_t src, n, fill, pad;
};
void mrg_launch_stage_scatter(const uint8_t *d_stage, uint32_t table_off, uint32_t nops, hipStream_t s);

#ifndef MRG_MAP_STEAL_K
#define MRG_MAP_STEAL_K 4        // blocks a wave takes from the pool at a time
#endif
#define MRG_WMAP_MAXB1 4096      // L1 buckets the wide map's LDS cursors hold
#define MRG_WIDE_IX1 260         // bytes of one partition's L1 splitter index (257 entries + prefix bits)
#define MRG_WMAP_IXR 64          // partitions whose index fits the wide map's LDS

// A set of keys with counts (SoA).  len > 16 keys have their bytes at heap[hoff .. hoff+len).
struct KeySet {
    uint64_t *k0, *k1, *cnt, *hoff;
    uint32_t *doc, *len, *part;
};

struct TableArgs {
    uint64_t *tk0, *tk1, *tcnt;
    uint32_t *tdoc;
    uint64_t cap;                // power of two
    uint32_t hash_bits;
};

// Exchange record, MRG_XREC_BYTES = 24 (include/mrgpu.h).  Short form (len <= 16): a, b = the packed
// key, v = count (wc; a count above MRG_XREC_VMAX goes out as several records, which the receiver
// sums) or the doc id (indexer).  Long form (len > 16): a = heap offset of the key bytes in the
// sender's heap segment, b = count (wc) / 1 (indexer), v = doc id (indexer) / MRG_EMPTY_DOC (wc).
struct XRec {
    uint64_t a, b;
    uint32_t v, len;
};
static_assert(sizeof(XRec) == 24, "XRec layout");
#define MRG_XREC_VMAX 0xFFFFFFFFull
// Records per key of the export: short wc keys carry at most vmax (MRG_XREC_VMAX; smaller only as a
// test knob) of their count per record
__host__ __device__ inline uint64_t mrg_xrec_per_key(uint64_t cnt, uint32_t len, bool indexer, uint64_t vmax) {
    return (indexer || len > 16u || cnt <= vmax) ? 1ull : (cnt + vmax - 1u) / vmax;
}

// Line record of the text reduce (k_text.hip -> mrg_reduce_text): one "key value" line of an
// intermediate file; keys longer than 16 bytes are addressed in place in the file buffer.
struct LRec {
    uint64_t k0, k1, cnt;
    uint32_t doc, len;
    uint64_t heap;
};
static_assert(sizeof(LRec) == 40, "LRec layout");

// Long items: keys > 16 bytes, as raw byte ranges of `base` (input text or a received heap).
struct LongItems {
    const uint8_t *base;
    uint64_t *start;
    uint32_t *rawlen, *doc;
    uint64_t *cnt;               // null: 1 each
    uint64_t n;
    int verbatim;                // 1: the ranges hold the key bytes exactly (exchange heap, text keys);
                                 // 0: raw token bytes, X-class codepoints are dropped (wc.rs:7-8)
};

// ---- k_map.hip
// `dev_args` is device memory for one MapArgs (the kernel reads its arguments from there)
// h: the args to copy to dev_args first (nullptr: already there)
void mrg_launch_map(const MapArgs *h, MapArgs *dev_args, int app, int grid, int lds_cap, hipStream_t s,
                    bool wide = false);
uint64_t mrg_map_tiles(uint64_t doc_lo, uint64_t doc_hi);  // wave blocks (NSUB KiB) of a document (16-B grid)
int mrg_map_cap(int app, int lds_cap);  // LDS-table entries per map workgroup actually used for lds_cap
int mrg_map_max_grid(int app, int lds_cap, int device);
// Dense long-token records from the map's per-workgroup regions and shared list (A as launched):
// region w's min(lcount[w], lper) records, then min(counters[CNT_LONGX], lovf) list records, to
// [0, n) of (start, len, doc); n = their total (on the device: counters[CNT_LONG] when nothing was lost).
void mrg_launch_long_compact(const MapArgs &A, int grid, uint64_t *start, uint32_t *len, uint32_t *doc,
                             hipStream_t s);
void mrg_launch_long_prep(const uint8_t *base, const uint64_t *start, const uint32_t *rawlen, uint64_t n,
                          uint64_t *k0, uint64_t *k1, uint32_t *flen, uint64_t *flen64, uint64_t *fp,
                          uint32_t hash_bits, int verbatim, hipStream_t s);
void mrg_launch_long_gather(const uint8_t *base, const uint64_t *start, const uint32_t *rawlen, uint64_t n,
                            const uint64_t *dst_off, uint8_t *heap, int verbatim, hipStream_t s);

// ---- k_keys.hip
struct BucketArgs {
    const uint64_t *pool;        // MapArgs::pool (MRG_TAIL_BYTES records) and pool16 (wc, 16-byte records)
    const uint64_t *rbase;
    const uint32_t *bcap, *bcount;
    const uint64_t *pool16;
    const uint64_t *rbase16;
    const uint32_t *bcap16, *bcount16;
    const uint64_t *movf;        // map-side overflow lists (MapArgs::ovf / onext / ocap)
    const uint32_t *monext;
    uint32_t mocap;
    const uint64_t *fk0, *fk1;
    const uint32_t *fcnt, *fdoc, *foff;
    uint32_t nreg, regcap;       // map workgroups (flush regions) and entries per region
    // keys that do not fit a bucket's LDS table (exact overflow, aggregated in the HBM table)
    uint64_t *ok0, *ok1;
    uint32_t *ocnt, *odoc;
    uint64_t ocap;
    KeySet out;
    unsigned long long *counters;
    uint32_t hash_bits;
    uint32_t ablate;             // timing only (MRG_AGG_ABLATE): 1 = no table adds, 2 = no hash either, 4 = no tail stream at all
    uint32_t nsub;               // workgroups per bucket, each summing one hash sub-range (1 = whole bucket)
    uint64_t kcap;               // capacity of `out` (keys beyond it are counted, not written)
    uint32_t n_reduce;           // partition of every key written (SipHash-1-3 % n_reduce; 0 = leave to k_partition)
};
// count32: the job has fewer than 2^32 tokens (32-bit LDS counts, a larger table); nreg <= 1024 then
void mrg_launch_bucket_agg(const BucketArgs &a, bool indexer, bool count32, hipStream_t s);
// wide (sort-based) aggregation of the map records, wc only (k_keys.hip)
struct SortRec;
void mrg_launch_wide_counts(const BucketArgs &a, uint64_t *cnt, uint64_t nseg, hipStream_t s);
void mrg_launch_wide_gather(const BucketArgs &a, const uint64_t *off, uint64_t nseg, uint32_t n_reduce, SortRec *out,
                            hipStream_t s);
void mrg_launch_wide_heads(const SortRec *r, uint64_t n, uint64_t *head, uint64_t *cv, hipStream_t s);
void mrg_launch_wide_keys(const SortRec *r, uint64_t n, const uint64_t *head, const uint64_t *E, KeySet ks,
                          uint64_t *F, hipStream_t s);
void mrg_launch_wide_cnt(const uint64_t *F, uint64_t runs, uint64_t n, const uint64_t *C, uint64_t ctot, KeySet ks,
                         hipStream_t s);
void mrg_launch_table_clear(const TableArgs &t, bool indexer, hipStream_t s);
void mrg_launch_table_insert(const TableArgs &t, const uint64_t *k0, const uint64_t *k1, const uint32_t *cnt32,
                             const uint32_t *doc, uint64_t n, bool indexer, hipStream_t s);
void mrg_launch_table_insert_x(const TableArgs &t, const XRec *x, uint64_t n, bool indexer, hipStream_t s);
void mrg_launch_table_insert_l(const TableArgs &t, const LRec *x, uint64_t n, bool indexer, hipStream_t s);
void mrg_launch_table_compact(const TableArgs &t, bool indexer, KeySet out, unsigned long long *counter,
                              hipStream_t s);
void mrg_launch_partition(KeySet ks, const uint8_t *heap, uint64_t n, uint32_t n_reduce, hipStream_t s);
void mrg_launch_long_group(const uint64_t *fp_sorted, const uint32_t *idx_sorted, const uint32_t *doc,
                           const uint8_t *heap, const uint64_t *hoff, const uint32_t *flen, uint64_t n,
                           uint32_t *rep, hipStream_t s);
void mrg_launch_long_emit(const uint32_t *rep, const uint64_t *cnt_in, const uint64_t *k0, const uint64_t *k1,
                          const uint32_t *flen, const uint64_t *hoff, const uint32_t *doc, uint64_t n,
                          unsigned long long *acc, KeySet out, unsigned long long *counter, bool indexer,
                          hipStream_t s);
void mrg_launch_x_split_long(const XRec *x, uint64_t n, const uint64_t *seg_rec_end, const uint64_t *seg_heap_base,
                             uint32_t n_segs, LongItems li, unsigned long long *counter, bool indexer, hipStream_t s);
void mrg_launch_l_split_long(const LRec *x, uint64_t n, const uint64_t *seg_rec_end, const uint64_t *seg_heap_base,
                             uint32_t n_segs, LongItems li, unsigned long long *counter, hipStream_t s);
void mrg_launch_export_count(KeySet ks, uint64_t n, uint32_t n_owners, unsigned long long *rec_cnt,
                             unsigned long long *heap_cnt, bool indexer, uint64_t vmax, hipStream_t s);
void mrg_launch_export_pack(KeySet ks, const uint8_t *heap, uint64_t n, uint32_t n_owners,
                            const uint64_t *rec_base, const uint64_t *heap_base, unsigned long long *rec_cur,
                            unsigned long long *heap_cur, XRec *out, uint8_t *out_heap, bool indexer, uint64_t vmax,
                            hipStream_t s);
// carry (wc, counts not changed after the sort): count and length in the record's doc / pad words
void mrg_launch_make_sortrec(KeySet ks, uint64_t n, const uint32_t *doc_rank, void *recs, hipStream_t s,
                             bool carry = false);
void mrg_launch_fill_u32(uint32_t *p, uint32_t v, uint64_t n, hipStream_t s);
void mrg_launch_fill_u64(uint64_t *p, uint64_t v, uint64_t n, hipStream_t s);
void mrg_launch_iota_u32(uint32_t *p, uint64_t n, hipStream_t s);

// ---- k_sort.hip
uint64_t mrg_scan_tmp_elems(uint64_t n);
// exclusive scan of u64 values (in == out allowed); tmp holds mrg_scan_tmp_elems(n) u64
void mrg_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, uint64_t *tmp, hipStream_t s);
// the same for u32 values (tmp: mrg_scan_tmp_elems(n) u32)
void mrg_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *tmp, hipStream_t s);
struct SortRec {  // 32 bytes
    uint64_t k0, k1;
    uint32_t part, doc;
    uint32_t idx, pad;
};
struct SortPlan {
    bool use_doc, use_k1, use_k0, use_part;
    uint32_t part_bytes;   // bytes of `part` that can be non-zero
    uint32_t doc_bytes;
};
uint64_t mrg_sort_tmp_bytes(uint64_t n);
// Stable sort by (part, k0, k1, doc) ascending.  Returns the buffer (recs or alt) with the result.
SortRec *mrg_radix_sort(SortRec *recs, SortRec *alt, uint64_t n, const SortPlan &plan, void *tmp, hipStream_t s,
                        int *passes_run);
// Sort by (part, k0, k1, doc) ascending, not stable (keys distinct): MSD buckets on (part: pbits
// significant bits, leading key bits) + LDS bitonic sort per bucket; oversized buckets by the LSD
// sort.  Returns recs or alt; *n_big = oversized buckets (more than 16: the whole array went through
// the LSD sort).
SortRec *mrg_msd_sort(SortRec *recs, SortRec *alt, uint64_t n, uint32_t pbits, const SortPlan &plan, void *tmp,
                      hipStream_t s, uint32_t *n_big, uint32_t *h_pinned);
// The same in two halves, with no host wait in between: _launch enqueues the MSD passes and an async
// copy of the oversized-bucket count into *h_nbig (pinned); once the stream has reached it, _finish
// sorts the oversized buckets (if any) and returns recs or alt like mrg_msd_sort.
void mrg_msd_sort_launch(SortRec *recs, SortRec *alt, uint64_t n, uint32_t pbits, void *tmp, hipStream_t s,
                         uint32_t *h_nbig);
SortRec *mrg_msd_sort_finish(SortRec *recs, SortRec *alt, uint64_t n, const SortPlan &plan, void *tmp, hipStream_t s,
                             uint32_t nb);
// Stable sort of (u64 key, u32 val) pairs by key, in place in (keys, vals); kv_tmp holds 4n u64.
void mrg_radix_sort_u64(uint64_t *keys, uint32_t *vals, uint64_t *kv_tmp, uint64_t n, void *tmp, hipStream_t s);

// ---- k_format.hip
struct FormatArgs {
    const SortRec *recs;        // sorted by (part, key prefix, doc rank)
    uint64_t n;
    KeySet ks;
    const uint8_t *heap;
    uint64_t heap_bytes;        // bytes of the long-key heap (bounds the wc output before it is sized)
    uint32_t n_reduce;
    int drop_last;
    int indexer;
    int any_long;
    int carried;                // wc: count and length carried in the records (mrg_launch_make_sortrec)
    const uint8_t *names;       // indexer: doc names concatenated in rank order
    const uint64_t *name_off;   // [n_docs + 1], by rank
};
// Writes every mr-{r}.txt (concatenated in r order) into *out_buf (grown from the pool) and the
// partition byte offsets to part_off_host[0..n_reduce].  Returns the total byte count.
uint64_t mrg_format(const FormatArgs &f, DevPool &pool, uint8_t **out_buf, uint64_t *out_cap,
                    uint64_t *part_off_host, hipStream_t s);
// Insertion-sort runs of equal (part, 16-byte prefix) that involve a long key by full key bytes.
void mrg_launch_fix_runs(SortRec *r, uint64_t n, KeySet ks, const uint8_t *heap, hipStream_t s);
// final.txt: part2[key] = 1 for the keys the per-partition pass drops (drop-last), else 0.
void mrg_launch_final_part(const SortRec *r, uint64_t n, KeySet ks, const uint8_t *heap, int drop_last,
                           uint32_t *part2, hipStream_t s);

// ---- k_text.hip: the reference's text intermediates (mr-{m}-{r}.txt)
struct TextTok {  // one token of a map task, input order
    uint64_t k0, k1, start;
    uint32_t rawlen, klen, part, pad;
};
uint64_t mrg_text_segments(uint64_t n);  // 64-byte segments (threads) over n bytes
void mrg_launch_text_tok(const uint8_t *in, uint64_t n, uint32_t n_reduce, const uint64_t *base, uint64_t *cnt,
                         TextTok *out, unsigned long long *err, hipStream_t s);
void mrg_launch_text_keys(const TextTok *t, uint64_t n, uint64_t *part, uint32_t *idx, hipStream_t s);
void mrg_launch_text_len(const TextTok *t, const uint32_t *idx, uint64_t n, uint64_t *L, hipStream_t s);
void mrg_launch_text_part_off(const uint64_t *part, const uint64_t *O, uint64_t n, uint32_t R, uint64_t total,
                              uint64_t *part_off, hipStream_t s);
void mrg_launch_text_write(const uint8_t *in, const TextTok *t, const uint32_t *idx, uint64_t n, const uint64_t *O,
                           uint8_t *out, hipStream_t s);
void mrg_launch_utf8_check(const uint8_t *in, uint64_t n, unsigned long long *err, hipStream_t s);
void mrg_launch_text_lines(const uint8_t *in, const uint64_t *fo, const uint64_t *fe, uint32_t nf, uint64_t nseg,
                           const uint64_t *base, uint64_t *cnt, LRec *out, unsigned long long *err,
                           unsigned long long *nempty, hipStream_t s);
void mrg_launch_add_first(const SortRec *r, KeySet ks, uint64_t v, hipStream_t s);

// ---- k_wide.hip: high-cardinality aggregation by a two-level sample sort
#define MRG_WIDE_T1 65536u       // records per L1 tile
#define MRG_WIDE_MAXB2 1024u     // leaves per L1 bucket; leaf id = bucket * MRG_WIDE_MAXB2 + j
struct WideLeafArgs {
    const uint64_t *kin;         // records in leaf order (2 words each)
    uint64_t *kout;              // distinct keys (2 words each) at leaf_out[leaf] + i
    const uint64_t *bstart;      // [B1 + 1]
    const uint32_t *nleaf;       // [B1]
    const uint64_t *leaf_lo, *leaf_lb;
    uint32_t B1r, R;
    const uint64_t *wk0, *wk1, *wcnt;  // weighted keys (flushed map tables), sorted by (part, key)
    const uint32_t *wpart;
    uint64_t nw;
    uint32_t maxd;               // 0 = default capacity
    uint64_t *ocnt;
    uint64_t *leaf_out;
    uint32_t *leaf_nd;
    uint64_t *leaf_bytes;
    uint32_t *leaf_last;
    uint32_t *ovf_list;
    unsigned long long *ovf_n;
    unsigned long long *nkeys;   // += distinct keys of every finished leaf
    uint64_t *wr;                // [B1 * MRG_WIDE_MAXB2][2] scratch: weighted-key range of each leaf
    unsigned long long *prof;    // diagnostics (builds with -DMRG_WIDE_PROF): leaf phase clocks [16]
    uint32_t *big_list;          // [B1 * MRG_WIDE_MAXB2] leaves passed from the one-wave to the workgroup kernel
    unsigned long long *big_n;   // their count (zeroed by the caller)
    uint32_t *leaf_pk;           // [B1 * MRG_WIDE_MAXB2] 1: the leaf's counts are packed into its key slots (zeroed by the caller)
    uint32_t pack;               // packing allowed: every count fits 32 bits (fewer than 2^32 tokens)
    const uint64_t *leaf_hi;     // [B1 * MAXB2] one past each leaf's last record in kin (L2 may leave gaps)
    const uint64_t *leaf_dlo;    // [B1 * MAXB2] each leaf's first record in the dense order (its output slots)
};
void mrg_wide_launch_counts(const BucketArgs &a, uint64_t *cnt_main, uint64_t *segptr, uint64_t *cnt_flush,
                            hipStream_t s);
void mrg_wide_launch_flush_gather(const BucketArgs &a, const uint64_t *off, uint64_t *k0, uint64_t *k1, uint32_t *c,
                                  hipStream_t s);
void mrg_wide_launch_sample1(const BucketArgs &a, const uint64_t *off, uint64_t nseg, uint64_t n, uint32_t S,
                             uint32_t R, SortRec *out, hipStream_t s);
void mrg_wide_launch_split1(const SortRec *smp, uint32_t S, uint32_t R, uint32_t B1r, uint64_t *spl, hipStream_t s);
size_t mrg_wide_l1_lds(uint32_t R, uint32_t B1r, uint32_t B1);
void mrg_wide_launch_l1(const BucketArgs &a, const uint64_t *off, const uint64_t *segptr, uint64_t nseg, uint64_t n,
                        const uint64_t *spl1, uint32_t R, uint32_t B1r, uint32_t *cnt, uint32_t ntiles, uint64_t *out,
                        uint16_t *bid, uint8_t *ix1, bool scatter, hipStream_t s);
void mrg_wide_launch_bstart(const uint32_t *cnt, uint32_t B1, uint32_t ntiles, uint64_t n, uint64_t *bstart,
                            hipStream_t s);
// The wide map's regions as L2 input (MapArgs::wrec / w12 / wl16 layout); rin == null: L1's output
struct WmapIn {
    const uint64_t *rin = nullptr;
    const uint32_t *soff = nullptr;  // [B1][grid + 2] segment starts (mrg_wmap_launch_seg)
    uint32_t grid = 0, wcap = 0, w12 = 0, wl16cap = 0;
    const uint64_t *wl16 = nullptr;
};
void mrg_wide_l2_prof(unsigned long long out[8]);
// sparse L2 leaves (the wide map's buckets only): out must hold 9 n / 4 + 16 records (bucket b's leaves in
// [9 bstart[b] / 4, 9 bstart[b + 1] / 4)); capacities capmul x sampled records + capadd (test knobs)
struct L2Sparse {
    bool on = false;
    uint32_t capmul = 6, capadd = 64;   // (r06 v11: 6 x the sampled records + 64, leaf target 256)
    uint32_t sample_min = 65536;      // records: smaller buckets histogram exactly
    uint32_t *redo_flags = nullptr;   // [B1], zeroed: buckets the exact second launch redoes
};
void mrg_wide_launch_l2(const uint64_t *in, uint64_t *out, const uint64_t *bstart, const uint64_t *spl1, uint32_t B1,
                        uint32_t B1r, uint32_t target, uint32_t *nleaf, uint64_t *leaf_lo, uint64_t *leaf_hi,
                        uint64_t *leaf_dlo, uint64_t *leaf_lb, uint16_t *sub, hipStream_t s,
                        const WmapIn &wm = WmapIn{}, const L2Sparse &sp = L2Sparse{});
// wide map (near-unique input): a sample of the input text's tokens (k_wsample_text), adjacent
// duplicates of the sorted sample, the L1 splitter index, the regions' per-bucket segment starts
void mrg_wide_launch_sample_text(const uint8_t *in, const uint64_t *doc_off, uint32_t n_docs, uint64_t total,
                                 uint32_t S, uint32_t R, SortRec *out, hipStream_t s);
void mrg_wide_launch_sample_dups(const SortRec *r, uint32_t S, unsigned long long *dups, hipStream_t s);
// the cold-context near-unique test: S (<= 8192) unsorted samples, dups[0] = repeats, dups[1] = 13..16-byte keys
void mrg_wide_launch_sample_uniq(const SortRec *r, uint32_t S, unsigned long long *dups, hipStream_t s);
void mrg_wide_launch_l1ix(const uint64_t *spl1, uint32_t R, uint32_t B1r, uint8_t *ix1, hipStream_t s);
// segment starts of bucket b: soff[b * (grid + 2) + w], w < grid the regions, w = grid the 16-byte list
// (wl16n null: empty), [grid + 1] the bucket's total, also in nb[b]
void mrg_wmap_launch_seg(const uint32_t *wcnt, uint32_t B1, uint32_t grid, uint32_t wcap, const uint32_t *wl16n,
                         uint32_t wl16cap, uint32_t *soff, uint64_t *nb, hipStream_t s);
void mrg_wide_launch_weights(const SortRec *r, uint64_t n, KeySet ks, uint64_t *wk0, uint64_t *wk1, uint64_t *wcnt,
                             uint32_t *wpart, hipStream_t s);
void mrg_wide_launch_leaf(const WideLeafArgs &w, uint32_t B1, hipStream_t s);
void mrg_wide_launch_fallback(const WideLeafArgs &w, const uint32_t *list, uint32_t nlist, DevPool &pool,
                              hipStream_t s);
void mrg_wide_launch_drop(const uint32_t *nleaf, uint32_t B1r, uint32_t R, const uint32_t *leaf_nd, uint64_t *leaf_bytes,
                          const uint32_t *leaf_last, uint32_t *leaf_drop, hipStream_t s);
void mrg_wide_launch_write(const uint64_t *keys, const uint64_t *ocnt, const uint32_t *leaf_pk, const uint32_t *nleaf,
                           const uint64_t *leaf_out, const uint32_t *leaf_nd, const uint32_t *leaf_drop,
                           const uint64_t *leaf_off, uint32_t B1, uint8_t *out, hipStream_t s);
void mrg_wide_launch_part_off(const uint64_t *leaf_off, uint32_t B1r, uint32_t R, uint64_t total, uint64_t *part_off,
                              hipStream_t s);
void mrg_wide_launch_dense(const uint64_t *keys, const uint64_t *ocnt, const uint32_t *leaf_pk, const uint64_t *leaf_out,
                           const uint32_t *leaf_nd, const uint32_t *dense_off, uint32_t B1, uint32_t B1r, KeySet ks,
                           hipStream_t s);

// ---- k_gen.hip
int mrg_gen_zipf_impl(uint8_t *dst, uint64_t n, uint64_t seed, uint64_t file_index, uint32_t vocab, double s, uint32_t style,
                      hipStream_t st);
int mrg_gen_unique_impl(uint8_t *dst, uint64_t n, uint64_t seed, uint64_t file_index, hipStream_t st);
