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
pub const MRG_FLAG_FINAL_TXT: u32 = 0x2;
pub const fn mrg_flag_debug_hash_bits(n: u32) -> u32 {
    (n & 0xFF) << 8
}
pub const MRG_XREC_BYTES: usize = 40;
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
    pub fn mrg_free(p: *mut c_void);

    pub fn mrg_gen_zipf(ctx: *mut mrg_ctx, d_dst: *mut u8, n_bytes: u64, seed: u64, file_index: u64, vocab: u32,
                        s: f64) -> c_int;
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

/// The whole job over `n_gpus` GPUs (mrcoordinator + workers): out_dir/mr-{r}.txt (+ final.txt).
pub fn run_job(files: &[&str], n_reduce: u32, app: c_int, out_dir: &str, flags: u32, n_gpus: i32)
               -> Result<(), Error> {
    let cs: Vec<CString> = files.iter().map(|f| CString::new(*f).unwrap()).collect();
    let ps: Vec<*const c_char> = cs.iter().map(|c| c.as_ptr()).collect();
    let od = CString::new(out_dir).unwrap();
    check(unsafe { mrg_run_job(ps.as_ptr(), ps.len(), n_reduce, app, od.as_ptr(), flags, n_gpus) })
}
