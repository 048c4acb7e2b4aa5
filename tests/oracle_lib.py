"""ctypes loader for the C oracle (oracle/build/liboracle.so) -- TEST INFRASTRUCTURE ONLY.

Loaded only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker.
"""
import ctypes
import os
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "liboracle.so")

FAITHFUL = 0
FAST = 1

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run `make -C oracle`)")
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_class.argtypes = [ctypes.c_uint32]
        L.oracle_class.restype = ctypes.c_int
        L.oracle_siphash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_siphash.restype = ctypes.c_uint64
        L.oracle_key_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_key_hash.restype = ctypes.c_uint64
        L.oracle_tokens.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(u8p),
                                    ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_validate_utf8.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_wc.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                ctypes.c_uint32, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(u8p),
                                ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_indexer.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(ctypes.c_char_p), ctypes.c_int, ctypes.c_uint32,
                                     ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_wc_workers.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_char_p,
                                         ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_wc_mt.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                   ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(u8p),
                                   ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_reduce_files.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(u8p),
                                          ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, rc):
        super().__init__(f"oracle error {rc}")
        self.rc = rc


def _take(ptr, n):
    data = ctypes.string_at(ptr, n)
    lib().oracle_free(ptr)
    return data


def tokens(data: bytes):
    L = lib()
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    rc = L.oracle_tokens(data, len(data), ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise OracleError(rc)
    s = _take(out, n.value)
    return [t for t in s.split(b"\n")[:-1]]


def key_hash(key: bytes) -> int:
    return lib().oracle_key_hash(key, len(key))


def siphash(data: bytes, c=1, d=3, k0=0, k1=0) -> int:
    return lib().oracle_siphash(data, len(data), c, d, k0, k1)


def _split(buf, offs, R):
    return [buf[offs[r]:offs[r + 1]] for r in range(R)]


def wc(files, n_reduce, mode=FAST, workdir=None):
    """Returns the list of mr-{r}.txt contents (bytes)."""
    L = lib()
    n = len(files)
    arr = (ctypes.c_char_p * max(n, 1))(*files)
    lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in files])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    offs = (ctypes.c_size_t * (n_reduce + 1))()
    tmp = None
    if mode == FAITHFUL and workdir is None:
        tmp = tempfile.TemporaryDirectory(prefix="oracle_wc_")
        workdir = tmp.name
    try:
        rc = L.oracle_wc(arr, lens, n, n_reduce, mode, workdir.encode() if workdir else None,
                         ctypes.byref(out), ctypes.byref(olen), offs)
    finally:
        if tmp is not None:
            tmp.cleanup()
    if rc:
        raise OracleError(rc)
    buf = _take(out, olen.value)
    return _split(buf, list(offs), n_reduce)


def indexer(files, docs, n_reduce):
    L = lib()
    n = len(files)
    arr = (ctypes.c_char_p * max(n, 1))(*files)
    lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in files])
    darr = (ctypes.c_char_p * max(n, 1))(*[d.encode() for d in docs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    offs = (ctypes.c_size_t * (n_reduce + 1))()
    rc = L.oracle_indexer(arr, lens, darr, n, n_reduce, ctypes.byref(out), ctypes.byref(olen), offs)
    if rc:
        raise OracleError(rc)
    buf = _take(out, olen.value)
    return _split(buf, list(offs), n_reduce)


def wc_workers(files, n_reduce, workers, workdir=None):
    """The reference structure (FAITHFUL tasks) on `workers` threads pulling map, then reduce tasks."""
    L = lib()
    n = len(files)
    arr = (ctypes.c_char_p * max(n, 1))(*files)
    lens = (ctypes.c_size_t * max(n, 1))(*[len(f) for f in files])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    offs = (ctypes.c_size_t * (n_reduce + 1))()
    with tempfile.TemporaryDirectory(prefix="oracle_wk_", dir=workdir) as d:
        rc = L.oracle_wc_workers(arr, lens, n, n_reduce, workers, d.encode(), ctypes.byref(out), ctypes.byref(olen),
                                 offs)
    if rc:
        raise OracleError(rc)
    return _split(_take(out, olen.value), list(offs), n_reduce)


def wc_mt(buffers, n_reduce, threads=8):
    """FAST mode on `threads` threads.  buffers: bytes / bytearray / numpy uint8 arrays (not copied)."""
    import numpy as np
    L = lib()
    arrs = [np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else b for b in buffers]
    n = len(arrs)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    lens = (ctypes.c_size_t * max(n, 1))(*[a.size for a in arrs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    olen = ctypes.c_size_t()
    offs = (ctypes.c_size_t * (n_reduce + 1))()
    rc = L.oracle_wc_mt(ptrs, lens, n, n_reduce, threads, ctypes.byref(out), ctypes.byref(olen), offs)
    if rc:
        raise OracleError(rc)
    return _split(_take(out, olen.value), list(offs), n_reduce)


def reduce_files(contents, r=0):
    """The FAITHFUL reduce task (worker.rs:157-193) over intermediate file contents: contents[m] is
    written to mr-{m}-{r}.txt in a scratch directory, then the oracle reads them back and reduces."""
    L = lib()
    with tempfile.TemporaryDirectory(prefix="oracle_rd_") as d:
        for m, c in enumerate(contents):
            with open(os.path.join(d, f"mr-{m}-{r}.txt"), "wb") as f:
                f.write(c)
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t()
        rc = L.oracle_reduce_files(d.encode(), len(contents), r, ctypes.byref(out), ctypes.byref(n))
    if rc:
        raise OracleError(rc)
    return _take(out, n.value)
