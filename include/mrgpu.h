/*
 * mrgpu.h -- C ABI of libmrgpu.so, the MI355X (gfx950) engine for the Freebirdgo/MapReduce_Rust
 * worker data path: map -> SipHash partition -> (shuffle) -> sort -> group/reduce -> mr-{r}.txt.
 *
 * Plain pointers and sizes only.  Every call returns MRG_OK (0) or a negative MRG_E* code and never
 * aborts across the ABI; mrg_last_error() gives a thread-local message for the last failure.
 * Device pointers ("d_") are HIP device allocations on the context's device; host pointers ("h_").
 *
 * Reference interfaces each entry point replaces (paths relative to the reference repo root):
 *   mrg_map        call_map_func(Box::new(wc::map), &contents)      src/mr/worker.rs:16-18, 147-150
 *                  + cal_hash_for_key / index = h % reduce_n        src/mr/worker.rs:111-115, 129
 *                  + write_key_value_to_file (partitioned output)   src/mr/worker.rs:117-140
 *                  wc::map                                          src/app/wc.rs:6-13
 *   mrg_reduce     read_file_to_mem_reduce + sort + group loop      src/mr/worker.rs:79-109, 157-193
 *                  call_reduce_func(Box::new(wc::reduce), ...)      src/mr/worker.rs:20-25, 174-178
 *                  wc::reduce                                       src/app/wc.rs:15-17
 *   mrg_run_job    the whole mrcoordinator + N x mrworker run       src/bin/mrworker.rs:43-149,
 *                  (static plan instead of coordinator.rs:137-215 task assignment), 1..8 GPUs
 *   mrg_job_shuffle the mr-{m}-{r}.txt hand-off between map and reduce workers through the shared
 *                  CWD (write_key_value_to_file worker.rs:117-140 -> read_file_to_mem_reduce
 *                  worker.rs:79-109), as one RCCL all-to-all over xGMI (owner of r = r % n_ranks)
 *   mrg_map_text   write_key_value_to_file, byte-exact mr-{m}-{r}.txt  src/mr/worker.rs:117-140
 *   mrg_reduce_text read_file_to_mem_reduce over mr-{m}-{r}.txt      src/mr/worker.rs:79-109, 157-193
 *   mrg_job_final  generate_output: cat mr-* | sort > final.txt     src/run.sh:16-20
 *   mrg_job_*      the same path with device-resident input, split at the shuffle so that a
 *                  multi-GPU host can exchange partitions between GPUs (RCCL all-to-all).
 */
#ifndef MRGPU_H
#define MRGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define MRG_OK 0
#define MRG_EINVAL (-1)   /* bad argument / state (reference: assert! failures, worker.rs:130,143-160) */
#define MRG_EUTF8 (-2)    /* input is not UTF-8 (reference: read_to_string().unwrap() panics, worker.rs:75) */
#define MRG_EHIP (-3)     /* HIP runtime error */
#define MRG_ENOMEM (-4)   /* device or host allocation failed */
#define MRG_EIO (-5)      /* file open/read/write failed (reference: unwrap/`?` on fs ops, worker.rs:73,122,168) */
#define MRG_ECOMM (-6)    /* RCCL communicator error, or another rank of the job failed */

/* ---- apps (the reference selects wc at compile time, worker.rs:5,148,175) ---- */
#define MRG_APP_WC 0       /* src/app/wc.rs */
#define MRG_APP_INDEXER 1  /* build-defined (no indexer in the reference): word -> "n doc1,doc2,..." */

/* ---- flags ---- */
#define MRG_FLAG_NO_COMPAT_DROP_LAST 0x1u  /* default (flag clear): reproduce worker.rs:169-184, which never
                                              writes the last group of a partition.  Set: write it. */
#define MRG_FLAG_FINAL_TXT 0x2u  /* mrg_run_job: also write out_dir/final.txt (src/run.sh:16-20) */
/* bits 8..15: truncate every internal (non-partition) hash to this many bits; 0 = full 64 bits.
   A test knob that forces hash collisions so the full-string tie-break paths are exercised. */
#define MRG_FLAG_DEBUG_HASH_BITS(n) (((uint32_t)(n) & 0xFFu) << 8)

/* Exchange record (mrg_job_export / mrg_job_import / mrg_parts): 24 bytes, little-endian.
 *   short key (len <= 16):
 *     u64 k0, k1   the key bytes, big-endian packed, zero padded (keys never contain NUL)
 *     u32 v        wc: occurrences (a key counted more than 0xFFFFFFFF times is sent as several records,
 *                  which the receiver sums); indexer: global document id
 *     u32 len      key length in bytes
 *   long key (len > 16):
 *     u64 heap     byte offset of the key bytes in the sender's heap segment
 *     u64 count    occurrences (wc) / 1 (indexer)
 *     u32 v        global document id (indexer), 0xFFFFFFFF (wc)
 *     u32 len      key length in bytes
 * The heap holds the bytes of keys longer than 16 bytes.  (Format 2; format 1 had 40-byte records.) */
#define MRG_XREC_BYTES 24

typedef struct mrg_ctx mrg_ctx;
typedef struct mrg_parts mrg_parts;

typedef struct {
    uint64_t input_bytes;      /* bytes mapped */
    uint64_t tokens;           /* tokens produced by the tokenizer */
    uint64_t long_tokens;      /* tokens longer than 16 bytes (slow path) */
    uint64_t map_records;      /* records leaving the map kernel (LDS-combine misses + flush) */
    uint64_t distinct_keys;    /* keys after aggregation (wc: words; indexer: (word, doc) pairs) */
    uint64_t output_bytes;     /* bytes of all mr-{r}.txt */
    double ms_map;             /* map kernel (tokenize + LDS combine), last call, HIP events */
    double ms_aggregate;       /* global aggregation + partition hash */
    double ms_sort;            /* radix sort */
    double ms_format;          /* output formatting */
    uint32_t map_launches;     /* map kernel launches in the last mrg_job_map */
    uint32_t agg_launches;     /* bucket-aggregation launches (> 1: its overflow list was regrown) */
    uint64_t overflow_keys;    /* records that took the exact HBM-table overflow path */
    double ms_exchange;        /* mrg_job_shuffle: the data send/recv group, HIP events on the ctx stream */
    uint64_t exchange_sent;    /* bytes this rank sent to peers (records + heap; its own slice excluded) */
    uint64_t exchange_recv;    /* bytes this rank received from peers */
    uint64_t map_spill;        /* map records that overflowed their tail region into a bucket's shared
                                  overflow list (last map launch) */
    uint64_t nonascii_tiles;   /* 1 KiB tiles that took the non-ASCII tokenizer (last map launch) */
    uint64_t tail_records_16;  /* wc: map records stored as 16-byte tail records (keys of 13..16 bytes; the
                                  others are 12-byte records); 0 for the indexer (all 24-byte records) */
    uint32_t spec_agg;         /* the aggregation queued behind the map: 0 none, 1 used, 2 dropped */
    uint32_t agg_path;         /* aggregation taken: 0 none, 1 bucket tables, 2 wide (sort-based) */
    uint32_t map_kind;         /* map kernel: 0 LDS combine + hash-bucketed tail records, 1 the wide map
                                  (near-unique keys: every key straight to its sort bucket) */
    uint32_t reserved;
} mrg_stats;

/* ABI history: 1 = round-1 layout; 2 = mrg_run_job's last argument is n_gpus (was a device index);
 * 3 = 24-byte exchange records (were 40), mrg_run_get_stats; 4 = mrg_stats gains nonascii_tiles,
 * tail_records_16, spec_agg, agg_path; 5 = mrg_stats gains map_kind, mrg_comm_count, mrg_pool_stats;
 * 6 = mrg_pool_alloc_stats.  mrg_version() names the ABI it implements. */
#define MRG_ABI_VERSION 6

const char *mrg_last_error(void);
const char *mrg_version(void);

/* One context per thread and device.  Owns a HIP stream (or uses one set by mrg_set_stream) and all
 * device workspaces, which grow on demand and are reused across jobs. */
int mrg_open(int device, mrg_ctx **out);
int mrg_close(mrg_ctx *ctx);
/* Run every kernel of this context on `hip_stream` (a hipStream_t; NULL = the context's own). */
int mrg_set_stream(mrg_ctx *ctx, void *hip_stream);
int mrg_get_stats(mrg_ctx *ctx, mrg_stats *out);
/* Per-stage HIP-event timing (mrg_stats.ms_*); off by default (it adds events to the stream). */
int mrg_set_timing(mrg_ctx *ctx, int enable);

/* ---- device-resident job (bench, multi-GPU) ---- */

/* Start a job.  n_reduce = nReduce (worker.rs:129).  Clears previous job state. */
int mrg_job_begin(mrg_ctx *ctx, int app, uint32_t n_reduce, uint32_t flags);
/* Document names, indexed by global document id (indexer output; ignored by wc).  Every rank of a
 * multi-GPU job passes the full table.  Names must not contain ' ', ',' or '\n'. */
int mrg_job_set_doc_names(mrg_ctx *ctx, const char *const *names, uint32_t n_names);
/* Input: documents laid out back to back in ONE device buffer d_bytes (16-byte aligned);
 * document i is d_bytes[h_doc_off[i] .. h_doc_off[i+1]) with global id h_doc_ids[i] (NULL: i).
 * The buffer is borrowed until the next mrg_job_begin. */
int mrg_job_set_input(mrg_ctx *ctx, const uint8_t *d_bytes, const uint64_t *h_doc_off, uint32_t n_docs,
                      const uint32_t *h_doc_ids);
/* Map: tokenize (wc.rs:6-13) + combine + SipHash partition (worker.rs:111-115).  Validates UTF-8. */
int mrg_job_map(mrg_ctx *ctx);
/* Shuffle boundary.  Owner of partition r is r % n_owners.  Sizes first (host arrays of n_owners),
 * then pack into caller device buffers ordered by owner (records, then heap bytes). */
int mrg_job_export_sizes(mrg_ctx *ctx, uint32_t n_owners, uint64_t *h_rec_counts, uint64_t *h_heap_bytes);
int mrg_job_export(mrg_ctx *ctx, void *d_rec, void *d_heap);
/* Replace the job's keys by the aggregation of received exchange records: the concatenation of
 * n_segs senders' exports, sender i contributing h_seg_recs[i] records and h_seg_heap[i] heap bytes
 * (record heap offsets are relative to their sender's heap segment).  n_segs = 0: one segment. */
int mrg_job_import(mrg_ctx *ctx, const void *d_rec, uint64_t n_rec, const void *d_heap, uint64_t heap_bytes,
                   const uint64_t *h_seg_recs, const uint64_t *h_seg_heap, uint32_t n_segs);
/* Reduce: sort (byte order, worker.rs:162-164), group, reduce, format every owned partition.
 * *h_out_bytes = total bytes of the mr-{r}.txt contents (concatenated in r order). */
int mrg_job_reduce(mrg_ctx *ctx, uint64_t *h_out_bytes);
/* Device pointer to the output and the byte offset of each partition (h_part_off[n_reduce + 1]). */
int mrg_job_output(mrg_ctx *ctx, const uint8_t **d_out, uint64_t *h_part_off);
/* Copy the output to host memory (h_dst of at least *h_out_bytes). */
int mrg_job_copy_output(mrg_ctx *ctx, uint8_t *h_dst, uint64_t cap);
/* final.txt of src/run.sh:16-20 (generate_output: cat mr-* | sort > final.txt, with LC_ALL=C), built
 * on the device from the job's keys: every line of every mr-{r}.txt this context holds, sorted
 * bytewise (= by key: key bytes are all > ' ').  *d_out stays valid until the next job call. */
int mrg_job_final(mrg_ctx *ctx, const uint8_t **d_out, uint64_t *h_bytes);
int mrg_job_copy_final(mrg_ctx *ctx, uint8_t *h_dst, uint64_t cap);

/* ---- multi-GPU: one rank per GPU, the shuffle as an RCCL all-to-all over xGMI ----
 * The reference moves map output to the reduce workers through mr-{m}-{r}.txt files in a shared
 * directory (worker.rs:117-140 -> :79-109) and hands out tasks on demand (coordinator.rs:137-215).
 * Here the plan is static: rank g maps its input shard, partition r is reduced by rank r % n_ranks,
 * and the hand-off is one exchange of combined per-key records. */
#define MRG_COMM_ID_BYTES 128
typedef struct mrg_comm mrg_comm;
/* A fresh communicator id (an RCCL unique id): made by one rank, given to every rank out of band. */
int mrg_comm_get_id(uint8_t id[MRG_COMM_ID_BYTES]);
/* Join the communicator as `rank` of n_ranks, on ctx's device.  Collective over the n_ranks callers
 * (they must call it concurrently: separate processes, or one thread per GPU). */
int mrg_comm_init(mrg_ctx *ctx, const uint8_t id[MRG_COMM_ID_BYTES], int n_ranks, int rank, mrg_comm **out);
int mrg_comm_destroy(mrg_comm *comm);
/* The exchange step, collective over the communicator, after mrg_job_map on every rank: the job's
 * keys are packed by owner (r % n_ranks), the per-owner counts go through an all-to-all, the records
 * and long-key heap bytes through grouped send/recv on the ctx stream, and the received records
 * replace the job's keys (mrg_job_import).  Then mrg_job_reduce formats the partitions this rank
 * owns (the others come out empty).  Every rank must reach this call: a rank whose map failed must
 * still tell the others (the host's concern; mrg_run_job does it). */
int mrg_job_shuffle(mrg_ctx *ctx, mrg_comm *comm);
/* Ranks of the communicator as RCCL counts them (ncclCommCount): the bench reports it beside n_gpus. */
int mrg_comm_count(const mrg_comm *comm, int *n_ranks);

/* ---- diagnostics ---- */
/* The context's device buffer pool: blocks handed out and not yet returned (between calls this is
 * the job state the context keeps), and all bytes it holds (handed out + cached).  Either may be NULL. */
int mrg_pool_stats(mrg_ctx *ctx, uint64_t *outstanding, uint64_t *held_bytes);
/* Device allocations the pool has made since mrg_open (cumulative): hipMalloc calls, their bytes and
 * the host milliseconds spent inside them.  A fresh context's first job pays these; later jobs reuse
 * cached blocks.  Either pointer may be NULL.  (ABI 6.) */
int mrg_pool_alloc_stats(mrg_ctx *ctx, uint64_t *n_allocs, uint64_t *alloc_bytes, double *alloc_ms);

/* ---- plugin-surface equivalents, host buffers (one map task / one reduce task) ---- */

/* One map task over one input file's bytes: wc.rs:6-13 + worker.rs:117-140, combined per
 * partition.  doc = the document name (indexer value); doc_id its global id. */
int mrg_map(mrg_ctx *ctx, int app, const uint8_t *h_bytes, size_t n, const char *doc, uint32_t doc_id,
            uint32_t n_reduce, uint32_t flags, mrg_parts **out);
/* Records of partition r of a map output (exchange-record format above). */
int mrg_parts_get(const mrg_parts *parts, uint32_t r, const uint8_t **h_rec, uint64_t *n_rec,
                  const uint8_t **h_heap, uint64_t *heap_bytes);
void mrg_parts_free(mrg_parts *parts);
/* One reduce task: partition r of k map outputs -> exact bytes of mr-{r}.txt (worker.rs:157-193).
 * For the indexer, doc_names[id] names global document id (n_docs entries). */
int mrg_reduce(mrg_ctx *ctx, int app, uint32_t r, const mrg_parts *const *in, size_t k, uint32_t n_reduce,
               uint32_t flags, const char *const *doc_names, uint32_t n_docs, uint8_t **h_out, size_t *h_out_len);

/* ---- the reference's text intermediates, byte for byte (wc) ---- */

/* One map task writing mr-{m}-{r}.txt exactly as Worker::write_key_value_to_file does
 * (src/mr/worker.rs:117-140): "{key} 1\n" for every token of wc::map (src/app/wc.rs:6-13) in input
 * order, into file r = SipHash-1-3(key) % n_reduce (worker.rs:111-115, 129).  *h_out receives the
 * n_reduce files' bytes concatenated (free with mrg_free); h_part_off[n_reduce + 1] their offsets. */
int mrg_map_text(mrg_ctx *ctx, const uint8_t *h_bytes, size_t n, uint32_t n_reduce, uint8_t **h_out,
                 uint64_t *h_part_off);
/* One reduce task over k intermediate files' contents (Worker::read_file_to_mem_reduce + reduce,
 * worker.rs:79-109, 157-193): UTF-8 checked (MRG_EUTF8), every non-empty line must be exactly
 * "key value" (MRG_EINVAL, the reference's assert!), values counted per key (wc.rs:15-17), keys in
 * byte order, the last group dropped unless MRG_FLAG_NO_COMPAT_DROP_LAST.  Returns mr-{r}.txt. */
int mrg_reduce_text(mrg_ctx *ctx, const uint8_t *const *h_files, const uint64_t *h_sizes, size_t k, uint32_t flags,
                    uint8_t **h_out, size_t *h_out_len);

/* The whole job (mrcoordinator + workers, mrworker.rs:43-149) on GPUs 0 .. n_gpus-1, one host thread
 * per GPU: GPU g reads and maps files m with m % n_gpus == g (the coordinator's map task ids,
 * coordinator.rs:137-176), the shuffle is mrg_job_shuffle, GPU g reduces and writes out_dir/mr-{r}.txt
 * for r % n_gpus == g (the reduce task ids, coordinator.rs:178-215).  With MRG_FLAG_FINAL_TXT also
 * out_dir/final.txt: each GPU sorts the lines it holds, the host merges the n_gpus sorted runs.
 * Indexer document names are the file paths as given (the reference opens "data/gut-{m}.txt").
 * Files are read by several host threads per GPU through pinned staging, overlapped with the copies
 * to the device.  Every phase runs on all GPUs and is joined before the next, and the exchange agrees
 * on every rank's status before each transfer: a failure on any GPU fails the call, never hangs it.
 * (ABI 2 changed the last argument from a device index to n_gpus.) */
int mrg_run_job(const char *const *files, size_t n_files, uint32_t n_reduce, int app, const char *out_dir,
                uint32_t flags, int n_gpus);

/* Wall-clock phases of the last mrg_run_job on the calling thread (host clock, milliseconds). */
typedef struct {
    double ms_total;        /* the whole call */
    double ms_open;         /* contexts + communicators */
    double ms_read;         /* input files -> device (read + H2D, overlapped; slowest GPU) */
    double ms_map;          /* map + aggregation after the read (slowest GPU) */
    double ms_shuffle;      /* the exchange (0 without a communicator) */
    double ms_reduce;       /* sort + format + D2H of the output (+ final.txt) */
    double ms_write;        /* mr-{r}.txt (+ final.txt) files */
    uint64_t input_bytes;
    uint64_t output_bytes;  /* bytes of all mr-{r}.txt */
    int n_gpus;
    double ms_map_alloc;    /* of ms_map: host time inside the fresh contexts' device allocations (slowest
                               GPU; every mrg_run_job opens fresh contexts, ABI 6) */
    double ms_map_kernel;       /* of ms_map: the map kernel (HIP events, slowest GPU; ABI 6) */
    double ms_aggregate_kernel; /* of ms_map: the aggregation after it (HIP events, slowest GPU; ABI 6) */
} mrg_run_stats;
int mrg_run_get_stats(mrg_run_stats *out);

/* Free host memory returned by the library (mrg_reduce / mrg_map_text / mrg_reduce_text output). */
void mrg_free(void *p);

/* ---- synthetic inputs for the benchmark (not on the data path) ---- */

/* Zipf(s) text over a vocabulary of `vocab` distinct lowercase words (BASELINE config C3/C4),
 * written to d_dst[0 .. n_bytes).  Deterministic in (seed, file_index); see DESIGN.md. */
int mrg_gen_zipf(mrg_ctx *ctx, uint8_t *d_dst, uint64_t n_bytes, uint64_t seed, uint64_t file_index,
                 uint32_t vocab, double s);
/* The same Zipf text in a given style: MRG_TEXT_ASCII (= mrg_gen_zipf) or MRG_TEXT_GUTENBERG (the
 * reference corpus's kind of Unicode: U+2019 apostrophes, U+201C/U+201D quotes, U+2014 dashes joining
 * words, Latin-1 letters; about one non-ASCII codepoint per 150 bytes). */
#define MRG_TEXT_ASCII 0
#define MRG_TEXT_GUTENBERG 1
int mrg_gen_text(mrg_ctx *ctx, uint8_t *d_dst, uint64_t n_bytes, uint64_t seed, uint64_t file_index,
                 uint32_t vocab, double s, uint32_t style);
/* Near-unique 12-character keys (BASELINE config C5): token i of file f, 1% repeats. */
int mrg_gen_unique(mrg_ctx *ctx, uint8_t *d_dst, uint64_t n_bytes, uint64_t seed, uint64_t file_index);

#ifdef __cplusplus
}
#endif
#endif /* MRGPU_H */
