"""ctypes binding of libmrgpu.so (include/mrgpu.h).  No CPU fallback: a missing library raises.

Every entry point of the C ABI is bound here with its exact signature; MrgError carries the
status code and mrg_last_error() text.  Device buffers are passed as raw device pointers (ints);
callers typically own them as torch CUDA tensors (plumbing only, never in the ABI).
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))

APP_WC = 0
APP_INDEXER = 1
FLAG_NO_COMPAT_DROP_LAST = 0x1
FLAG_FINAL_TXT = 0x2
XREC_BYTES = 24  # include/mrgpu.h MRG_XREC_BYTES (ABI 3)
ABI_VERSION = 6  # include/mrgpu.h MRG_ABI_VERSION

OK, EINVAL, EUTF8, EHIP, ENOMEM, EIO, ECOMM = 0, -1, -2, -3, -4, -5, -6
_CODES = {EINVAL: "EINVAL", EUTF8: "EUTF8", EHIP: "EHIP", ENOMEM: "ENOMEM", EIO: "EIO", ECOMM: "ECOMM"}
COMM_ID_BYTES = 128


def debug_hash_bits(n):
    """MRG_FLAG_DEBUG_HASH_BITS(n): truncate internal hashes to n bits (forces collisions)."""
    return (n & 0xFF) << 8


def kernel_source_sha():
    """sha256 over the sources libmrgpu.so is built from (kernels, headers, host layer): keys the
    committed PMC traffic figure (profiles/map_traffic.json) to the code it was measured on."""
    import hashlib
    d = os.path.join(_HERE, "csrc")
    h = hashlib.sha256()
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".h", ".inc", ".cpp")) and f != "mrgpu_cli.cpp":
            h.update(f.encode())
            h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def lib_path():
    return os.environ.get("MRG_LIB", os.path.join(_HERE, "lib", "libmrgpu.so"))


class MrgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{_CODES.get(code, code)}: {msg}")
        self.code = code


class Stats(C.Structure):
    _fields_ = [("input_bytes", C.c_uint64), ("tokens", C.c_uint64), ("long_tokens", C.c_uint64),
                ("map_records", C.c_uint64), ("distinct_keys", C.c_uint64), ("output_bytes", C.c_uint64),
                ("ms_map", C.c_double), ("ms_aggregate", C.c_double), ("ms_sort", C.c_double),
                ("ms_format", C.c_double), ("map_launches", C.c_uint32), ("agg_launches", C.c_uint32),
                ("overflow_keys", C.c_uint64), ("ms_exchange", C.c_double), ("exchange_sent", C.c_uint64),
                ("exchange_recv", C.c_uint64), ("map_spill", C.c_uint64),
                ("nonascii_tiles", C.c_uint64), ("tail_records_16", C.c_uint64), ("spec_agg", C.c_uint32),
                ("agg_path", C.c_uint32), ("map_kind", C.c_uint32), ("reserved", C.c_uint32)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class RunStats(C.Structure):
    """mrg_run_stats: wall-clock phases of the last mrg_run_job on this thread."""
    _fields_ = [("ms_total", C.c_double), ("ms_open", C.c_double), ("ms_read", C.c_double), ("ms_map", C.c_double),
                ("ms_shuffle", C.c_double), ("ms_reduce", C.c_double), ("ms_write", C.c_double),
                ("input_bytes", C.c_uint64), ("output_bytes", C.c_uint64), ("n_gpus", C.c_int),
                ("ms_map_alloc", C.c_double), ("ms_map_kernel", C.c_double), ("ms_aggregate_kernel", C.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None
_vp = C.c_void_p
_u8p = C.POINTER(C.c_uint8)
_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)

_SIGS = {
    "mrg_last_error": (C.c_char_p, []),
    "mrg_version": (C.c_char_p, []),
    "mrg_open": (C.c_int, [C.c_int, C.POINTER(_vp)]),
    "mrg_close": (C.c_int, [_vp]),
    "mrg_set_stream": (C.c_int, [_vp, _vp]),
    "mrg_get_stats": (C.c_int, [_vp, C.POINTER(Stats)]),
    "mrg_set_timing": (C.c_int, [_vp, C.c_int]),
    "mrg_job_begin": (C.c_int, [_vp, C.c_int, C.c_uint32, C.c_uint32]),
    "mrg_job_set_doc_names": (C.c_int, [_vp, C.POINTER(C.c_char_p), C.c_uint32]),
    "mrg_job_set_input": (C.c_int, [_vp, _vp, _u64p, C.c_uint32, _u32p]),
    "mrg_job_map": (C.c_int, [_vp]),
    "mrg_job_export_sizes": (C.c_int, [_vp, C.c_uint32, _u64p, _u64p]),
    "mrg_job_export": (C.c_int, [_vp, _vp, _vp]),
    "mrg_job_import": (C.c_int, [_vp, _vp, C.c_uint64, _vp, C.c_uint64, _u64p, _u64p, C.c_uint32]),
    "mrg_job_reduce": (C.c_int, [_vp, _u64p]),
    "mrg_job_output": (C.c_int, [_vp, C.POINTER(_vp), _u64p]),
    "mrg_job_copy_output": (C.c_int, [_vp, _vp, C.c_uint64]),
    "mrg_job_final": (C.c_int, [_vp, C.POINTER(_vp), _u64p]),
    "mrg_job_copy_final": (C.c_int, [_vp, _vp, C.c_uint64]),
    "mrg_map": (C.c_int, [_vp, C.c_int, C.c_char_p, C.c_size_t, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32,
                          C.POINTER(_vp)]),
    "mrg_parts_get": (C.c_int, [_vp, C.c_uint32, C.POINTER(_vp), _u64p, C.POINTER(_vp), _u64p]),
    "mrg_parts_free": (None, [_vp]),
    "mrg_reduce": (C.c_int, [_vp, C.c_int, C.c_uint32, C.POINTER(_vp), C.c_size_t, C.c_uint32, C.c_uint32,
                             C.POINTER(C.c_char_p), C.c_uint32, C.POINTER(_vp), C.POINTER(C.c_size_t)]),
    "mrg_map_text": (C.c_int, [_vp, C.c_char_p, C.c_size_t, C.c_uint32, C.POINTER(_vp), _u64p]),
    "mrg_reduce_text": (C.c_int, [_vp, C.POINTER(C.c_char_p), _u64p, C.c_size_t, C.c_uint32, C.POINTER(_vp),
                                  C.POINTER(C.c_size_t)]),
    "mrg_run_job": (C.c_int, [C.POINTER(C.c_char_p), C.c_size_t, C.c_uint32, C.c_int, C.c_char_p, C.c_uint32,
                              C.c_int]),
    "mrg_run_get_stats": (C.c_int, [C.POINTER(RunStats)]),
    "mrg_comm_get_id": (C.c_int, [_vp]),
    "mrg_comm_init": (C.c_int, [_vp, _vp, C.c_int, C.c_int, C.POINTER(_vp)]),
    "mrg_comm_destroy": (C.c_int, [_vp]),
    "mrg_job_shuffle": (C.c_int, [_vp, _vp]),
    "mrg_comm_count": (C.c_int, [_vp, C.POINTER(C.c_int)]),
    "mrg_pool_stats": (C.c_int, [_vp, _u64p, _u64p]),
    "mrg_pool_alloc_stats": (C.c_int, [_vp, _u64p, _u64p, C.POINTER(C.c_double)]),
    "mrg_free": (None, [_vp]),
    "mrg_gen_zipf": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_double]),
    "mrg_gen_unique": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64]),
    "mrg_gen_text": (C.c_int, [_vp, _vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_double, C.c_uint32]),
}


def load():
    """Load libmrgpu.so and bind every exported entry point (raises if it is missing)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: when torch (the device-memory / stream / torch.distributed
        # plumbing) is present, import it first so libmrgpu.so binds to the libamdhip64.so.7 torch
        # already mapped (same soname) instead of loading a second runtime beside it.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"libmrgpu.so not built ({path}); run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(path)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def _check(rc):
    if rc != OK:
        raise MrgError(rc, load().mrg_last_error().decode(errors="replace"))


def _u64arr(xs):
    return (C.c_uint64 * max(len(xs), 1))(*xs)


class Parts:
    """One map task's output (mrg_parts): per-partition exchange records + long-key heap."""

    def __init__(self, handle, n_reduce):
        self.h = handle
        self.n_reduce = n_reduce

    def get(self, r):
        L = load()
        rec, heap = _vp(), _vp()
        nrec, nheap = C.c_uint64(), C.c_uint64()
        _check(L.mrg_parts_get(self.h, r, C.byref(rec), C.byref(nrec), C.byref(heap), C.byref(nheap)))
        return (C.string_at(rec, nrec.value * XREC_BYTES) if nrec.value else b"",
                C.string_at(heap, nheap.value) if nheap.value else b"")

    def free(self):
        if self.h:
            load().mrg_parts_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Context:
    """One mrg_ctx: a device, a stream, device workspaces, and the current job."""

    def __init__(self, device=0):
        L = load()
        h = _vp()
        _check(L.mrg_open(device, C.byref(h)))
        self.h = h
        self.device = device
        self.n_reduce = 0

    def close(self):
        if self.h:
            load().mrg_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_stream(self, stream_ptr):
        _check(load().mrg_set_stream(self.h, stream_ptr))

    def pool_stats(self):
        """mrg_pool_stats: (device blocks handed out and not returned, bytes the pool holds)."""
        n, b = C.c_uint64(), C.c_uint64()
        _check(load().mrg_pool_stats(self.h, C.byref(n), C.byref(b)))
        return n.value, b.value

    def pool_alloc_stats(self):
        """mrg_pool_alloc_stats: (hipMalloc calls, bytes, host ms spent in them) since the context opened."""
        n, b, ms = C.c_uint64(), C.c_uint64(), C.c_double()
        _check(load().mrg_pool_alloc_stats(self.h, C.byref(n), C.byref(b), C.byref(ms)))
        return n.value, b.value, ms.value

    def set_timing(self, on=True):
        _check(load().mrg_set_timing(self.h, 1 if on else 0))

    def stats(self):
        s = Stats()
        _check(load().mrg_get_stats(self.h, C.byref(s)))
        return s.as_dict()

    # ---- device-resident job
    def job_begin(self, app, n_reduce, flags=0):
        _check(load().mrg_job_begin(self.h, app, n_reduce, flags))
        self.n_reduce = n_reduce

    def set_doc_names(self, names):
        arr = (C.c_char_p * max(len(names), 1))(*[n.encode() for n in names])
        _check(load().mrg_job_set_doc_names(self.h, arr, len(names)))

    def set_input(self, dev_ptr, doc_off, doc_ids=None):
        if len(doc_off) < 1:
            raise ValueError("doc_off needs n_docs + 1 entries (at least [0])")
        n = len(doc_off) - 1
        off = _u64arr(doc_off)
        ids = (C.c_uint32 * max(n, 1))(*doc_ids) if doc_ids is not None else None
        _check(load().mrg_job_set_input(self.h, dev_ptr, off, n, ids))

    def map(self):
        _check(load().mrg_job_map(self.h))

    def export_sizes(self, n_owners):
        rec = (C.c_uint64 * n_owners)()
        heap = (C.c_uint64 * n_owners)()
        _check(load().mrg_job_export_sizes(self.h, n_owners, rec, heap))
        return list(rec), list(heap)

    def export(self, d_rec, d_heap):
        _check(load().mrg_job_export(self.h, d_rec, d_heap))

    def import_(self, d_rec, n_rec, d_heap, heap_bytes, seg_recs=None, seg_heap=None):
        if seg_recs is None:
            _check(load().mrg_job_import(self.h, d_rec, n_rec, d_heap, heap_bytes, None, None, 0))
        else:
            _check(load().mrg_job_import(self.h, d_rec, n_rec, d_heap, heap_bytes, _u64arr(seg_recs),
                                         _u64arr(seg_heap), len(seg_recs)))

    def shuffle(self, comm):
        """mrg_job_shuffle: the exchange over RCCL (collective over comm's ranks)."""
        _check(load().mrg_job_shuffle(self.h, comm.h))

    def reduce(self):
        n = C.c_uint64()
        _check(load().mrg_job_reduce(self.h, C.byref(n)))
        return n.value

    def output(self):
        d = _vp()
        off = (C.c_uint64 * (self.n_reduce + 1))()
        _check(load().mrg_job_output(self.h, C.byref(d), off))
        return d.value, list(off)

    def copy_output(self):
        _, off = self.output()
        buf = C.create_string_buffer(max(off[-1], 1))
        _check(load().mrg_job_copy_output(self.h, buf, off[-1]))
        return buf.raw[:off[-1]], off

    def copy_output_to(self, host_ptr, n):
        """mrg_job_copy_output into caller memory (e.g. a pinned buffer) of at least n bytes."""
        _check(load().mrg_job_copy_output(self.h, C.c_void_p(host_ptr), n))

    def outputs(self):
        """mr-{r}.txt contents for every partition r."""
        data, off = self.copy_output()
        return [data[off[r]:off[r + 1]] for r in range(self.n_reduce)]

    def final(self):
        """final.txt (src/run.sh:16-20, LC_ALL=C) of this job, built on the device."""
        d = _vp()
        n = C.c_uint64()
        _check(load().mrg_job_final(self.h, C.byref(d), C.byref(n)))
        buf = C.create_string_buffer(max(n.value, 1))
        _check(load().mrg_job_copy_final(self.h, buf, n.value))
        return buf.raw[:n.value]

    # ---- plugin surface (host buffers)
    def map_task(self, app, data, doc, doc_id, n_reduce, flags=0):
        h = _vp()
        _check(load().mrg_map(self.h, app, data, len(data), doc.encode(), doc_id, n_reduce, flags, C.byref(h)))
        return Parts(h, n_reduce)

    def reduce_task(self, app, r, parts, n_reduce, flags=0, doc_names=()):
        arr = (_vp * max(len(parts), 1))(*[p.h for p in parts])
        names = (C.c_char_p * max(len(doc_names), 1))(*[n.encode() for n in doc_names])
        out = _vp()
        n = C.c_size_t()
        _check(load().mrg_reduce(self.h, app, r, arr, len(parts), n_reduce, flags, names, len(doc_names),
                                 C.byref(out), C.byref(n)))
        data = C.string_at(out, n.value) if n.value else b""
        load().mrg_free(out)
        return data

    # ---- the reference's text intermediates (wc)
    def map_text(self, data, n_reduce):
        """mr-{m}-{r}.txt contents of one map task (worker.rs:117-140), for r < n_reduce."""
        out = _vp()
        off = (C.c_uint64 * (n_reduce + 1))()
        _check(load().mrg_map_text(self.h, data, len(data), n_reduce, C.byref(out), off))
        blob = C.string_at(out, off[n_reduce]) if off[n_reduce] else b""
        load().mrg_free(out)
        return [blob[off[r]:off[r + 1]] for r in range(n_reduce)]

    def reduce_text(self, files, flags=0):
        """mr-{r}.txt from the contents of the intermediate files mr-{m}-{r}.txt (worker.rs:79-109)."""
        arr = (C.c_char_p * max(len(files), 1))(*files)
        sizes = _u64arr([len(f) for f in files])
        out = _vp()
        n = C.c_size_t()
        _check(load().mrg_reduce_text(self.h, arr, sizes, len(files), flags, C.byref(out), C.byref(n)))
        data = C.string_at(out, n.value) if n.value else b""
        load().mrg_free(out)
        return data

    # ---- synthetic inputs (bench)
    def gen_zipf(self, dev_ptr, n_bytes, seed, file_index, vocab=1 << 20, s=1.1):
        _check(load().mrg_gen_zipf(self.h, dev_ptr, n_bytes, seed, file_index, vocab, s))

    def gen_text(self, dev_ptr, n_bytes, seed, file_index, vocab=1 << 20, s=1.1, style=1):
        """style 0: ASCII (= gen_zipf); 1: Gutenberg-like Unicode (MRG_TEXT_GUTENBERG)."""
        _check(load().mrg_gen_text(self.h, dev_ptr, n_bytes, seed, file_index, vocab, s, style))

    def gen_unique(self, dev_ptr, n_bytes, seed, file_index):
        _check(load().mrg_gen_unique(self.h, dev_ptr, n_bytes, seed, file_index))


def run_job(files, n_reduce, app=APP_WC, out_dir=".", flags=0, n_gpus=1):
    """mrg_run_job: the whole job over files on disk; returns its phase timings (mrg_run_get_stats)."""
    arr = (C.c_char_p * max(len(files), 1))(*[f.encode() for f in files])
    _check(load().mrg_run_job(arr, len(files), n_reduce, app, out_dir.encode(), flags, n_gpus))
    st = RunStats()
    _check(load().mrg_run_get_stats(C.byref(st)))
    return st.as_dict()


def merge_sorted_lines(runs):
    """The host k-way merge of per-GPU sorted final.txt runs (test entry, no GPU needed)."""
    L = load()
    f = L.mrg_test_merge_sorted_lines
    f.restype = C.c_int
    f.argtypes = [C.POINTER(C.c_char_p), _u64p, C.c_size_t, C.POINTER(_vp), _u64p]
    arr = (C.c_char_p * max(len(runs), 1))(*runs)
    out, n = _vp(), C.c_uint64()
    _check(f(arr, _u64arr([len(r) for r in runs]), len(runs), C.byref(out), C.byref(n)))
    data = C.string_at(out, n.value) if n.value else b""
    L.mrg_free(out)
    return data


def comm_id():
    """A fresh RCCL communicator id (bytes) for Comm(); made by one rank, shared out of band."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(load().mrg_comm_get_id(buf))
    return buf.raw


class Comm:
    """mrg_comm: this rank's membership of an RCCL communicator (one per GPU / context)."""

    def __init__(self, ctx, uid, n_ranks, rank):
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("communicator id must be %d bytes" % COMM_ID_BYTES)
        h = _vp()
        _check(load().mrg_comm_init(ctx.h, uid, n_ranks, rank, C.byref(h)))
        self.h = h
        self.n_ranks = n_ranks
        self.rank = rank

    def count(self):
        """mrg_comm_count: ranks of the RCCL communicator (ncclCommCount)."""
        n = C.c_int()
        _check(load().mrg_comm_count(self.h, C.byref(n)))
        return n.value

    def close(self):
        if self.h:
            _check(load().mrg_comm_destroy(self.h))
            self.h = None
