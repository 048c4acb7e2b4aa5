#!/bin/bash
# r06: where the k_map launch's end spread sits -- per workgroup: start, last wave's main-loop end, end
# (lib_variants/prof = -DMRG_MAP_PROF), C3 and zipf_u at 10 GiB, pool on and off.
mkdir -p gpurun_out/ph2
for w in zipf zipf_u; do
  for d in 16; do
    MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/prof/libmrgpu.so MRG_PROF=1 MRG_MAP_STEAL=$d timeout -k 10 200 python -u bench.py \
      --workload $w --steps 2 --warmup 1 --quick > gpurun_out/ph2/${w}_$d.log 2>&1 || exit 1
    echo "== $w pool 1/$d"; grep -E "phase clocks|map workgroups|flush steps" gpurun_out/ph2/${w}_$d.log | tail -3
  done
done
