"""Helpers for GPU tests: device staging through torch (plumbing only) and the libmrgpu job API."""
import torch

import mapreduce_rust_amd as M


def to_device(blobs, align=16):
    """Lay documents back to back in one device buffer; returns (tensor, doc_off)."""
    off = [0]
    for b in blobs:
        off.append(off[-1] + len(b))
    buf = bytearray(off[-1] + 64)
    for b, o in zip(blobs, off):
        buf[o:o + len(b)] = b
    t = torch.frombuffer(buf, dtype=torch.uint8).to("cuda:0")
    assert t.data_ptr() % align == 0
    return t, off


def run_wc(ctx, blobs, n_reduce, app=M.APP_WC, flags=0, names=None, doc_ids=None):
    t, off = to_device(blobs)
    ctx.job_begin(app, n_reduce, flags)
    if app == M.APP_INDEXER:
        ctx.set_doc_names(names)
    ctx.set_input(t.data_ptr(), off, doc_ids)
    ctx.map()
    ctx.reduce()
    outs = ctx.outputs()
    torch.cuda.synchronize()
    del t
    return outs
