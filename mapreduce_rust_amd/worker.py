"""Host-side mirror of the reference Worker (src/mr/worker.rs) over libmrgpu.so.

Same task structure and file conventions as the reference:
  Worker(map_n, reduce_n)                     worker.rs:28-37
  Worker.map(m):    data/gut-{m}.txt  ->  mr-{m}-{r}.txt for r < reduce_n     worker.rs:142-155
  Worker.reduce(r): mr-{m}-{r}.txt for m < map_n  ->  mr-{r}.txt              worker.rs:157-193
intermediates="text" (default, wc): mr-{m}-{r}.txt byte-identical to the reference's ("key 1" per
token in input order, mrg_map_text / mrg_reduce_text), so GPU and reference CPU workers can take
each other's tasks.  intermediates="records": the engine's combined form, mr-{m}-{r}.rec (per-key
counts as 24-byte exchange records + long-key heap, include/mrgpu.h; a 32-byte little-endian header
{u64 magic "MRGREC\\0\\0", u32 format, u32 record bytes, u64 n_records, u64 heap_bytes}, then the records
and the heap) -- far smaller, and the only form for the indexer.  mr-{r}.txt is
byte-identical to the reference's either way.  A map task and a reduce task may run in different
processes, as in the reference (the files in the working directory are the hand-off).
"""
import os
import struct

from . import native

APPS = {"wc": native.APP_WC, "indexer": native.APP_INDEXER}


REC_MAGIC = b"MRGREC\0\0"
REC_FORMAT = 2            # the exchange-record format of include/mrgpu.h (24-byte records, ABI >= 3)
_REC_HDR = struct.Struct("<8sIIQQ")


class RecFileError(ValueError):
    pass


def read_rec(path):
    """(records, heap) of an mr-{m}-{r}.rec file; raises RecFileError on a foreign, stale-format or
    truncated file (the import would otherwise read past what the file holds)."""
    with open(path, "rb") as f:
        hdr = f.read(_REC_HDR.size)
        if len(hdr) != _REC_HDR.size:
            raise RecFileError(f"{path}: truncated header")
        magic, fmt, xb, n, hb = _REC_HDR.unpack(hdr)
        if magic != REC_MAGIC:
            raise RecFileError(f"{path}: not an mrgpu record file")
        if fmt != REC_FORMAT or xb != native.XREC_BYTES:
            raise RecFileError(f"{path}: record format {fmt} ({xb}-byte records), expected {REC_FORMAT} "
                               f"({native.XREC_BYTES}-byte records)")
        # sizes from the header are checked against the file before anything is read (a corrupt
        # header must not make the reader allocate n * xb bytes)
        if _REC_HDR.size + n * xb + hb != os.fstat(f.fileno()).st_size:
            raise RecFileError(f"{path}: size does not match its header ({n} records, {hb} heap bytes)")
        rec = f.read(n * xb)
        heap = f.read(hb)
        if len(rec) != n * xb or len(heap) != hb or f.read(1):
            raise RecFileError(f"{path}: size does not match its header ({n} records, {hb} heap bytes)")
    return rec, heap


def write_rec(path, rec, heap):
    with open(path, "wb") as f:
        f.write(_REC_HDR.pack(REC_MAGIC, REC_FORMAT, native.XREC_BYTES, len(rec) // native.XREC_BYTES, len(heap)))
        f.write(rec)
        f.write(heap)


def _rec_path(m, r, cwd):
    return os.path.join(cwd, f"mr-{m}-{r}.rec")


def _txt_path(m, r, cwd):
    return os.path.join(cwd, f"mr-{m}-{r}.txt")      # worker.rs:120


class Worker:
    def __init__(self, map_n, reduce_n, app="wc", device=0, flags=0, cwd=".", intermediates=None):
        if app not in APPS:
            raise ValueError(f"unknown app {app!r}")
        if intermediates is None:
            intermediates = "text" if app == "wc" else "records"
        if intermediates not in ("text", "records") or (intermediates == "text" and app != "wc"):
            raise ValueError(f"intermediates={intermediates!r} not available for app {app!r}")
        self.map_n, self.reduce_n = map_n, reduce_n
        self.app = APPS[app]
        self.flags = flags
        self.cwd = cwd
        self.text = intermediates == "text"
        self.ctx = native.Context(device)

    def doc_name(self, m):
        return f"data/gut-{m}.txt"      # worker.rs:67

    def map(self, m):
        """Map task m: the input file's bytes -> per-partition records."""
        with open(os.path.join(self.cwd, self.doc_name(m)), "rb") as f:   # worker.rs:73-75
            data = f.read()
        if self.text:
            for r, blob in enumerate(self.ctx.map_text(data, self.reduce_n)):
                with open(_txt_path(m, r, self.cwd), "wb") as f:
                    f.write(blob)
            return True
        parts = self.ctx.map_task(self.app, data, self.doc_name(m), m, self.reduce_n, self.flags)
        try:
            for r in range(self.reduce_n):                                 # worker.rs:120-125
                rec, heap = parts.get(r)
                write_rec(_rec_path(m, r, self.cwd), rec, heap)
        finally:
            parts.free()
        return True

    def reduce(self, r):
        """Reduce task r: every map task's records of partition r -> mr-{r}.txt."""
        if self.text:
            files = []
            for m in range(self.map_n):                                    # worker.rs:84-93
                with open(_txt_path(m, r, self.cwd), "rb") as f:
                    files.append(f.read())
            out = self.ctx.reduce_text(files, self.flags)
            with open(os.path.join(self.cwd, f"mr-{r}.txt"), "wb") as f:   # worker.rs:167-168
                f.write(out)
            return True
        recs, heaps, seg_r, seg_h = [], [], [], []
        for m in range(self.map_n):                                        # worker.rs:84-107
            rec, heap = read_rec(_rec_path(m, r, self.cwd))
            recs.append(rec)
            heaps.append(heap)
            seg_r.append(len(rec) // native.XREC_BYTES)
            seg_h.append(len(heap))
        out = self._reduce_records(r, b"".join(recs), b"".join(heaps), seg_r, seg_h)
        with open(os.path.join(self.cwd, f"mr-{r}.txt"), "wb") as f:       # worker.rs:167-168
            f.write(out)
        return True

    def _reduce_records(self, r, rec, heap, seg_r, seg_h):
        import torch
        dev = torch.device("cuda", self.ctx.device)
        d_rec = torch.frombuffer(bytearray(rec) + bytearray(16), dtype=torch.uint8).to(dev)
        d_heap = torch.frombuffer(bytearray(heap) + bytearray(16), dtype=torch.uint8).to(dev)
        self.ctx.job_begin(self.app, self.reduce_n, self.flags)
        if self.app == native.APP_INDEXER:
            self.ctx.set_doc_names([self.doc_name(m) for m in range(self.map_n)])
        self.ctx.import_(d_rec.data_ptr(), sum(seg_r), d_heap.data_ptr(), sum(seg_h), seg_r, seg_h)
        self.ctx.reduce()
        return self.ctx.outputs()[r]

    def close(self):
        self.ctx.close()
