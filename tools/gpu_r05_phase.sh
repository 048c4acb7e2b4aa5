#!/bin/bash
# r05: k_map phase clocks (-DMRG_MAP_PROF variant) and ablations (-DMRG_MAP_ABLATION variant) on 2 GiB
# of C3 and zipf_u.
mkdir -p gpurun_out
for w in ${WORKLOADS:-zipf zipf_u}; do
  echo "== $w"
  MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/prof/libmrgpu.so BENCH_ARGS="--workload $w" bash tools/gpu_phase.sh || exit $?
  MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/abl/libmrgpu.so BENCH_ARGS="--workload $w" ABLATE_SET="${ABLATE_SET:-0 32 64 4 3 1}" bash tools/gpu_ablate.sh || exit $?
done
