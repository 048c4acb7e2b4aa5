"""CPU tests of the C ABI boundary: libmrgpu.so loads, exports every entry point declared in
include/mrgpu.h, the Python binding covers them all, and errors come back as status codes (no GPU
here: mrg_open must fail cleanly, never abort)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "mrgpu.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*(mrg_\w+)\s*\(", src, re.M)))


def test_header_declares_the_boundary():
    fns = header_functions()
    for f in ["mrg_open", "mrg_close", "mrg_map", "mrg_reduce", "mrg_run_job", "mrg_free", "mrg_last_error",
              "mrg_job_begin", "mrg_job_map", "mrg_job_export", "mrg_job_import", "mrg_job_reduce"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    import mapreduce_rust_amd as M
    lib = ctypes.CDLL(M.lib_path())
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    from mapreduce_rust_amd import native
    assert sorted(native.exported_symbols()) == header_functions()
    native.load()


def test_no_gpu_is_a_clean_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import mapreduce_rust_amd as M
    with pytest.raises(M.MrgError) as ei:
        M.Context(0)
    assert ei.value.code == -3
    assert M.native.load().mrg_version().startswith(b"mrgpu")


def test_record_layout_constant():
    src = open(os.path.join(ROOT, "include", "mrgpu.h")).read()
    assert "#define MRG_XREC_BYTES 24" in src and "#define MRG_ABI_VERSION 6" in src
    from mapreduce_rust_amd import native, shuffle
    assert native.XREC_BYTES == shuffle.XREC == 24 and native.ABI_VERSION == 6
    assert b"abi 6" in native.load().mrg_version()
    rs = open(os.path.join(ROOT, "mrgpu-sys", "src", "lib.rs")).read()
    assert "pub const MRG_XREC_BYTES: usize = 24;" in rs and "pub const MRG_ABI_VERSION: u32 = 6;" in rs


def test_merge_sorted_lines_host():
    """The host k-way merge of the GPUs' sorted final.txt runs (mrgpu.cpp merge_sorted_lines, the
    multi-GPU half of run.sh:16-20 `cat mr-* | sort`): equals sorted() of all lines, byte order (C
    locale), with runs lacking a final newline, equal prefixes, duplicates across runs and empty runs."""
    import random
    from mapreduce_rust_amd import native
    rng = random.Random(7)
    alpha = [b"a", b"b", b"ab", b"abc", b"z", b"\xc3\xa9", b"_", b"0"]
    for trial in range(200):
        lines = [b"".join(rng.choice(alpha) for _ in range(rng.randint(1, 4))) + b" " + str(rng.randint(1, 99)).encode()
                 for _ in range(rng.randint(0, 40))]
        k = rng.randint(1, 9)
        runs = [[] for _ in range(k)]
        for ln in lines:
            runs[rng.randrange(k)].append(ln)
        blobs = []
        for r in runs:
            r.sort()
            b = b"".join(x + b"\n" for x in r)
            if b and rng.random() < 0.3:
                b = b[:-1]  # no final newline
            blobs.append(b)
        got = native.merge_sorted_lines(blobs)
        assert got == b"".join(x + b"\n" for x in sorted(lines)), trial
    assert native.merge_sorted_lines([]) == b"" and native.merge_sorted_lines([b"", b""]) == b""
    assert native.merge_sorted_lines([b"ab 1\nb 2", b"a 3\nab 0\n"]) == b"a 3\nab 0\nab 1\nb 2\n"


def test_rust_ffi_crate_declares_the_header():
    """mrgpu-sys/src/lib.rs (not compiled here: no Rust toolchain) declares every entry point of
    include/mrgpu.h with the same number of parameters, and mrg_stats with the same fields."""
    hdr = open(os.path.join(ROOT, "include", "mrgpu.h")).read()
    rs = open(os.path.join(ROOT, "mrgpu-sys", "src", "lib.rs")).read()
    decl_c = {m.group(1): m.group(2) for m in re.finditer(r"^\s*(?:int|void|const char \*)\s*(mrg_\w+)\s*\(([^)]*)\)",
                                                         hdr, re.M)}
    decl_rs = {m.group(1): m.group(2) for m in re.finditer(r"pub fn (mrg_\w+)\(([^)]*)\)", rs, re.S)}
    assert sorted(decl_c) == sorted(k for k in decl_rs if k in decl_c) == header_functions()

    def arity(args):
        a = args.strip()
        return 0 if a in ("", "void") else a.count(",") + 1
    for f, args in decl_c.items():
        assert arity(args) == arity(decl_rs[f]), f
    stats_c = re.findall(r"^\s+(?:uint64_t|uint32_t|double)\s+(\w+);", hdr.split("} mrg_stats;")[0], re.M)
    stats_rs = re.findall(r"pub (\w+): (?:u64|u32|f64),", rs.split("pub struct mrg_stats")[1].split("}")[0])
    assert stats_c == stats_rs


def test_rec_file_header_checks(tmp_path):
    """mr-{m}-{r}.rec (worker.py, intermediates="records"): magic + format + record size in the header;
    a stale 16-byte-header file, a wrong format and a truncated body are refused before any import."""
    import struct
    from mapreduce_rust_amd import native, worker as W
    X = native.XREC_BYTES
    p = str(tmp_path / "mr-0-0.rec")
    rec, heap = bytes(range(X)) * 3, b"abcdefghijklmnopq"
    W.write_rec(p, rec, heap)
    assert W.read_rec(p) == (rec, heap)
    with open(p, "wb") as f:                                   # the round-3 layout: <u64 n, u64 heap>
        f.write(struct.pack("<QQ", 3, len(heap)) + rec + heap)
    with pytest.raises(W.RecFileError, match="not an mrgpu record file"):
        W.read_rec(p)
    with open(p, "wb") as f:
        f.write(struct.pack("<8sIIQQ", W.REC_MAGIC, 1, 40, 3, 0) + bytes(120))
    with pytest.raises(W.RecFileError, match="record format 1"):
        W.read_rec(p)
    W.write_rec(p, rec, heap)
    data = open(p, "rb").read()
    for cut in (10, len(data) - 1):
        with open(p, "wb") as f:
            f.write(data[:cut])
        with pytest.raises(W.RecFileError):
            W.read_rec(p)
    with open(p, "wb") as f:                                   # a corrupt count: refused before any read
        f.write(struct.pack("<8sIIQQ", W.REC_MAGIC, W.REC_FORMAT, X, 1 << 60, 0) + rec)
    with pytest.raises(W.RecFileError, match="does not match"):
        W.read_rec(p)
    with open(p, "wb") as f:
        f.write(data + b"x")
    with pytest.raises(W.RecFileError, match="does not match"):
        W.read_rec(p)
