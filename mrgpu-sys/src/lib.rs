//! Raw bindings of `include/mrgpu.h` (libmrgpu.so, hand-written HIP for gfx950) plus a thin safe
//! wrapper for the two calls the reference's `Worker` makes (src/mr/worker.rs:142-193).
//!
//! Every function returns `MRG_OK` (0) or a negative `MRG_E*` code; `mrg_last_error()` holds a
//! thread-local message.  Nothing aborts across the boundary.
#![allow(non_camel_case_types)]

use std::ffi::{c_char, c_int, c_void, CStr, CString};

pub const MRG_OK: c_int = 0;
pub const MRG_EINVAL: c_int = -1;
pub const MRG_EUTF8: c_int = -2;
pub const MRG_EHIP: c_int = -3;
pub const MRG_ENOMEM: c_int = -4;
pub const MRG_EIO: c_int = -5;
pub const MRG_ECOMM: c_int = -6;

pub const MRG_APP_WC: c_int = 0;
pub const MRG_APP_INDEXER: c_int = 1;

pub const MRG_FLAG_NO_COMPAT_DROP_LAST: u32 = 0x1;
pub const MRG_TEXT_ASCII: u32 = 0;
pub const MRG_TEXT_GUTENBERG: u32 = 1;
pub const MRG_FLAG_FINAL_TXT: u32 = 0x2;
pub const fn mrg_flag_debug_hash_bits(n: u32) -> u32 {
    (n & 0xFF) << 8
}
pub const MRG_XREC_BYTES: usize = 24;
pub const MRG_ABI_VERSION: u32 = 6;
pub const MRG_COMM_ID_BYTES: usize = 128;

#[repr(C)]
pub struct mrg_ctx {
    _p: [u8; 0],
}
#[repr(C)]
pub struct mrg_parts {
    _p: [u8; 0],
}
#[repr(C)]
pub struct mrg_comm {
    _p: [u8; 0],
}

#[repr(C)]
#[derive(Debug, Default, Clone, Copy)]
pub struct mrg_stats {
    pub input_bytes: u64,
    pub tokens: u64,
    pub long_tokens: u64,
    pub map_records: u64,
    pub distinct_keys: u64,
    pub output_bytes: u64,
    pub ms_map: f64,
    pub ms_aggregate: f64,
    pub ms_sort: f64,
    pub ms_format: f64,
    pub map_launches: u32,
    pub agg_launches: u32,
    pub overflow_keys: u64,
    pub ms_exchange: f64,
    pub exchange_sent: u64,
    pub exchange_recv: u64,
    pub map_spill: u64,
    pub nonascii_tiles: u64,
    pub tail_records_16: u64,
    pub spec_agg: u32,
    pub agg_path: u32,
    pub map_kind: u32,
    pub reserved: u32,
}

#[repr(C)]
#[derive(Debug, Default, Clone, Copy)]
pub struct mrg_run_stats {
    pub ms_total: f64,
    pub ms_open: f64,
    pub ms_read: f64,
    pub ms_map: f64,
    pub ms_shuffle: f64,
    pub ms_reduce: f64,
    pub ms_write: f64,
    pub input_bytes: u64,
    pub output_bytes: u64,
    pub n_gpus: c_int,
    pub ms_map_alloc: f64,
    pub ms_map_kernel: f64,
    pub ms_aggregate_kernel: f64,
}

extern "C" {
    pub fn mrg_last_error() -> *const c_char;
    pub fn mrg_version() -> *const c_char;
    pub fn mrg_open(device: c_int, out: *mut *mut mrg_ctx) -> c_int;
    pub fn mrg_close(ctx: *mut mrg_ctx) -> c_int;
    pub fn mrg_set_stream(ctx: *mut mrg_ctx, hip_stream: *mut c_void) -> c_int;
    pub fn mrg_get_stats(ctx: *mut mrg_ctx, out: *mut mrg_stats) -> c_int;
    pub fn mrg_set_timing(ctx: *mut mrg_ctx, enable: c_int) -> c_int;

    pub fn mrg_job_begin(ctx: *mut mrg_ctx, app: c_int, n_reduce: u32, flags: u32) -> c_int;
    pub fn mrg_job_set_doc_names(ctx: *mut mrg_ctx, names: *const *const c_char, n_names: u32) -> c_int;
    pub fn mrg_job_set_input(ctx: *mut mrg_ctx, d_bytes: *const u8, h_doc_off: *const u64, n_docs: u32,
                             h_doc_ids: *const u32) -> c_int;
    pub fn mrg_job_map(ctx: *mut mrg_ctx) -> c_int;
    pub fn mrg_job_export_sizes(ctx: *mut mrg_ctx, n_owners: u32, h_rec_counts: *mut u64,
                                h_heap_bytes: *mut u64) -> c_int;
    pub fn mrg_job_export(ctx: *mut mrg_ctx, d_rec: *mut c_void, d_heap: *mut c_void) -> c_int;
    pub fn mrg_job_import(ctx: *mut mrg_ctx, d_rec: *const c_void, n_rec: u64, d_heap: *const c_void,
                          heap_bytes: u64, h_seg_recs: *const u64, h_seg_heap: *const u64, n_segs: u32) -> c_int;
    pub fn mrg_job_reduce(ctx: *mut mrg_ctx, h_out_bytes: *mut u64) -> c_int;
    pub fn mrg_job_output(ctx: *mut mrg_ctx, d_out: *mut *const u8, h_part_off: *mut u64) -> c_int;
    pub fn mrg_job_copy_output(ctx: *mut mrg_ctx, h_dst: *mut u8, cap: u64) -> c_int;
    pub fn mrg_job_final(ctx: *mut mrg_ctx, d_out: *mut *const u8, h_bytes: *mut u64) -> c_int;
    pub fn mrg_job_copy_final(ctx: *mut mrg_ctx, h_dst: *mut u8, cap: u64) -> c_int;

    pub fn mrg_comm_get_id(id: *mut u8) -> c_int;
    pub fn mrg_comm_init(ctx: *mut mrg_ctx, id: *const u8, n_ranks: c_int, rank: c_int,
                         out: *mut *mut mrg_comm) -> c_int;
    pub fn mrg_comm_destroy(comm: *mut mrg_comm) -> c_int;
    pub fn mrg_job_shuffle(ctx: *mut mrg_ctx, comm: *mut mrg_comm) -> c_int;
    pub fn mrg_comm_count(comm: *const mrg_comm, n_ranks: *mut c_int) -> c_int;

    pub fn mrg_pool_stats(ctx: *mut mrg_ctx, outstanding: *mut u64, held_bytes: *mut u64) -> c_int;
    pub fn mrg_pool_alloc_stats(ctx: *mut mrg_ctx, n_allocs: *mut u64, alloc_bytes: *mut u64, alloc_ms: *mut f64) -> c_int;

    pub fn mrg_map(ctx: *mut mrg_ctx, app: c_int, h_bytes: *const u8, n: usize, doc: *const c_char, doc_id: u32,
                   n_reduce: u32, flags: u32, out: *mut *mut mrg_parts) -> c_int;
    pub fn mrg_parts_get(parts: *const mrg_parts, r: u32, h_rec: *mut *const u8, n_rec: *mut u64,
                         h_heap: *mut *const u8, heap_bytes: *mut u64) -> c_int;
    pub fn mrg_parts_free(parts: *mut mrg_parts);
    pub fn mrg_reduce(ctx: *mut mrg_ctx, app: c_int, r: u32, parts: *const *const mrg_parts, k: usize,
                      n_reduce: u32, flags: u32, doc_names: *const *const c_char, n_docs: u32,
                      h_out: *mut *mut u8, h_out_len: *mut usize) -> c_int;

    pub fn mrg_map_text(ctx: *mut mrg_ctx, h_bytes: *const u8, n: usize, n_reduce: u32, h_out: *mut *mut u8,
                        h_part_off: *mut u64) -> c_int;
    pub fn mrg_reduce_text(ctx: *mut mrg_ctx, h_files: *const *const u8, h_sizes: *const u64, k: usize,
                           flags: u32, h_out: *mut *mut u8, h_out_len: *mut usize) -> c_int;

    pub fn mrg_run_job(files: *const *const c_char, n_files: usize, n_reduce: u32, app: c_int,
                       out_dir: *const c_char, flags: u32, n_gpus: c_int) -> c_int;
    pub fn mrg_run_get_stats(out: *mut mrg_run_stats) -> c_int;
    pub fn mrg_free(p: *mut c_void);

    pub fn mrg_gen_zipf(ctx: *mut mrg_ctx, d_dst: *mut u8, n_bytes: u64, seed: u64, file_index: u64, vocab: u32,
                        s: f64) -> c_int;
    pub fn mrg_gen_text(ctx: *mut mrg_ctx, d_dst: *mut u8, n_bytes: u64, seed: u64, file_index: u64, vocab: u32,
                        s: f64, style: u32) -> c_int;
    pub fn mrg_gen_unique(ctx: *mut mrg_ctx, d_dst: *mut u8, n_bytes: u64, seed: u64, file_index: u64) -> c_int;
}

/// The library's last error message on this thread.
pub fn last_error() -> String {
    unsafe { CStr::from_ptr(mrg_last_error()).to_string_lossy().into_owned() }
}

#[derive(Debug)]
pub struct Error {
    pub code: c_int,
    pub msg: String,
}

impl std::fmt::Display for Error {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        write!(f, "mrgpu error {}: {}", self.code, self.msg)
    }
}
impl std::error::Error for Error {}

fn check(rc: c_int) -> Result<(), Error> {
    if rc == MRG_OK { Ok(()) } else { Err(Error { code: rc, msg: last_error() }) }
}

/// One map task's output (per-partition combined records).
pub struct Parts(*mut mrg_parts);
impl Drop for Parts {
    fn drop(&mut self) {
        unsafe { mrg_parts_free(self.0) }
    }
}
unsafe impl Send for Parts {}

/// A GPU context: one per worker thread and device (`Worker` holds one).
pub struct Ctx(*mut mrg_ctx);
impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { mrg_close(self.0) };
    }
}
unsafe impl Send for Ctx {}

impl Ctx {
    pub fn open(device: i32) -> Result<Ctx, Error> {
        let mut c = std::ptr::null_mut();
        check(unsafe { mrg_open(device, &mut c) })?;
        Ok(Ctx(c))
    }

    /// `call_map_func(wc::map, contents)` + `cal_hash_for_key` + the partition loop
    /// (src/mr/worker.rs:142-155): the input's per-partition records.
    pub fn map(&self, app: c_int, contents: &str, doc: &str, doc_id: u32, n_reduce: u32) -> Result<Parts, Error> {
        let d = CString::new(doc).map_err(|_| Error { code: MRG_EINVAL, msg: "NUL in doc name".into() })?;
        let mut p = std::ptr::null_mut();
        check(unsafe {
            mrg_map(self.0, app, contents.as_ptr(), contents.len(), d.as_ptr(), doc_id, n_reduce, 0, &mut p)
        })?;
        Ok(Parts(p))
    }

    /// Start a device-resident job (`mrg_job_begin`).
    pub fn job_begin(&self, app: c_int, n_reduce: u32, flags: u32) -> Result<(), Error> {
        check(unsafe { mrg_job_begin(self.0, app, n_reduce, flags) })
    }

    /// Input already in device memory: documents back to back from `d_bytes` (16-byte aligned),
    /// document i = bytes [doc_off[i], doc_off[i + 1]) (`mrg_job_set_input`).
    ///
    /// # Safety
    /// `d_bytes` must be a device allocation on this context's device holding `doc_off[n]` bytes, and
    /// stay valid until the next `job_begin`.
    pub unsafe fn job_set_input(&self, d_bytes: *const u8, doc_off: &[u64], doc_ids: Option<&[u32]>)
                                -> Result<(), Error> {
        let n = doc_off.len().saturating_sub(1) as u32;
        let ids = doc_ids.map_or(std::ptr::null(), |v| v.as_ptr());
        check(mrg_job_set_input(self.0, d_bytes, doc_off.as_ptr(), n, ids))
    }

    /// Map + combine + partition (`mrg_job_map`; wc.rs:6-13, worker.rs:111-131).
    pub fn job_map(&self) -> Result<(), Error> {
        check(unsafe { mrg_job_map(self.0) })
    }

    /// The exchange with the other ranks of `comm` (`mrg_job_shuffle`, RCCL over xGMI).
    pub fn shuffle(&self, comm: &Comm) -> Result<(), Error> {
        check(unsafe { mrg_job_shuffle(self.0, comm.0) })
    }

    /// Sort + group + reduce + format (`mrg_job_reduce`); then the bytes of every `mr-{r}.txt`,
    /// concatenated in r order, with the partition offsets (n_reduce + 1 of them).
    pub fn job_reduce(&self, n_reduce: u32) -> Result<(Vec<u8>, Vec<u64>), Error> {
        let mut total = 0u64;
        check(unsafe { mrg_job_reduce(self.0, &mut total) })?;
        let mut off = vec![0u64; n_reduce as usize + 1];
        check(unsafe { mrg_job_output(self.0, std::ptr::null_mut(), off.as_mut_ptr()) })?;
        let mut out = vec![0u8; total as usize];
        check(unsafe { mrg_job_copy_output(self.0, out.as_mut_ptr(), total) })?;
        Ok((out, off))
    }

    /// Counters and stage times of the last job (`mrg_get_stats`).
    pub fn stats(&self) -> Result<mrg_stats, Error> {
        let mut st = mrg_stats::default();
        check(unsafe { mrg_get_stats(self.0, &mut st) })?;
        Ok(st)
    }

    /// `Worker::reduce` (src/mr/worker.rs:157-193): the exact bytes of `mr-{r}.txt`.
    pub fn reduce(&self, app: c_int, r: u32, parts: &[Parts], n_reduce: u32, doc_names: &[&str])
                  -> Result<Vec<u8>, Error> {
        let ptrs: Vec<*const mrg_parts> = parts.iter().map(|p| p.0 as *const _).collect();
        let names: Vec<CString> = doc_names.iter().map(|n| CString::new(*n).unwrap()).collect();
        let name_ptrs: Vec<*const c_char> = names.iter().map(|n| n.as_ptr()).collect();
        let (mut out, mut len) = (std::ptr::null_mut(), 0usize);
        check(unsafe {
            mrg_reduce(self.0, app, r, ptrs.as_ptr(), ptrs.len(), n_reduce, 0, name_ptrs.as_ptr(),
                       name_ptrs.len() as u32, &mut out, &mut len)
        })?;
        let v = unsafe { std::slice::from_raw_parts(out, len) }.to_vec();
        unsafe { mrg_free(out as *mut c_void) };
        Ok(v)
    }
}

/// One rank's membership of an RCCL communicator (one process or thread per GPU).
pub struct Comm(*mut mrg_comm);
impl Drop for Comm {
    fn drop(&mut self) {
        unsafe { mrg_comm_destroy(self.0) };
    }
}
unsafe impl Send for Comm {}

impl Comm {
    /// A fresh communicator id, made by one rank and handed to the others out of band.
    pub fn new_id() -> Result<[u8; MRG_COMM_ID_BYTES], Error> {
        let mut id = [0u8; MRG_COMM_ID_BYTES];
        check(unsafe { mrg_comm_get_id(id.as_mut_ptr()) })?;
        Ok(id)
    }

    /// Join as `rank` of `n_ranks` on `ctx`'s device (collective: every rank calls it concurrently).
    pub fn init(ctx: &Ctx, id: &[u8; MRG_COMM_ID_BYTES], n_ranks: i32, rank: i32) -> Result<Comm, Error> {
        let mut m = std::ptr::null_mut();
        check(unsafe { mrg_comm_init(ctx.0, id.as_ptr(), n_ranks, rank, &mut m) })?;
        Ok(Comm(m))
    }
}

/// The whole job over `n_gpus` GPUs (mrcoordinator + workers): out_dir/mr-{r}.txt (+ final.txt);
/// returns the call's phase timings.
pub fn run_job(files: &[&str], n_reduce: u32, app: c_int, out_dir: &str, flags: u32, n_gpus: i32)
               -> Result<mrg_run_stats, Error> {
    let cs: Vec<CString> = files.iter().map(|f| CString::new(*f).unwrap()).collect();
    let ps: Vec<*const c_char> = cs.iter().map(|c| c.as_ptr()).collect();
    let od = CString::new(out_dir).unwrap();
    check(unsafe { mrg_run_job(ps.as_ptr(), ps.len(), n_reduce, app, od.as_ptr(), flags, n_gpus) })?;
    let mut st = mrg_run_stats::default();
    check(unsafe { mrg_run_get_stats(&mut st) })?;
    Ok(st)
}
