#!/bin/bash
# r06: k_map phase clocks and workgroup end times (lib_variants/prof = -DMRG_MAP_PROF) on C3 and zipf_u,
# 2 GiB and the full 10 GiB.
mkdir -p gpurun_out/ph
for w in zipf zipf_u; do
  for f in 8 40; do
    MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/prof/libmrgpu.so MRG_PROF=1 timeout -k 10 200 python -u bench.py --workload $w \
      --files-per-gpu $f --steps 2 --warmup 1 --quick > gpurun_out/ph/${w}_$f.log 2>&1 || exit $?
    echo "== $w $f files"; grep -E "phase clocks|map workgroups" gpurun_out/ph/${w}_$f.log | tail -2; grep "step:" gpurun_out/ph/${w}_$f.log | tail -1
  done
done
