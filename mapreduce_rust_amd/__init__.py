"""mapreduce_rust_amd -- MI355X-native engine for the Freebirdgo/MapReduce_Rust worker data path.

The compute path is libmrgpu.so (hand-written HIP for gfx950, C ABI in include/mrgpu.h).  This
package is the host-side mirror of the reference's interfaces over that ABI:

  mapreduce_rust_amd.native   ctypes binding of every entry point of include/mrgpu.h
  mapreduce_rust_amd.worker   Worker.map / Worker.reduce with the reference's file conventions
                              (src/mr/worker.rs: data/gut-{m}.txt -> mr-{r}.txt)
  mapreduce_rust_amd.shuffle  multi-GPU static plan: the library's own RCCL exchange (mrg_job_shuffle)
                              for one process per GPU, and a torch.distributed (gloo) exchange of the
                              same export/import records for host-staged rehearsals and CPU tests

There is no CPU fallback: if the HIP library is missing or no GPU is present, calls raise.
"""
from .native import (APP_INDEXER, APP_WC, FLAG_FINAL_TXT, FLAG_NO_COMPAT_DROP_LAST, Comm, Context, MrgError,
                     comm_id, debug_hash_bits, lib_path, load)

__all__ = ["APP_WC", "APP_INDEXER", "FLAG_NO_COMPAT_DROP_LAST", "FLAG_FINAL_TXT", "MrgError", "Context", "Comm",
           "comm_id", "debug_hash_bits", "lib_path", "load"]
