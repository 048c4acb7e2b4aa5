#!/bin/bash
# Map workgroup start/end spread (MRG_PROF=1 with the -DMRG_MAP_PROF variant in lib_variants/prof).
mkdir -p gpurun_out
MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/prof/libmrgpu.so MRG_PROF=1 timeout -k 10 200 python -u bench.py \
  --steps 3 --warmup 1 --quick ${BENCH_ARGS} > gpurun_out/wgspan.log 2>&1 || exit $?
grep -E "phase clocks|workgroups|step:" gpurun_out/wgspan.log | tail -9
