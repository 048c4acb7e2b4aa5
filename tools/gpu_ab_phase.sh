#!/bin/bash
# Map A/B of lib_variants (C3, then zipf_u), then the -DMRG_MAP_PROF variant's phase clocks on both.
VARIANTS="${VARIANTS_C3:-lib_variants/v31 lib}" STEPS=6 bash tools/gpu_ab.sh || exit $?
VARIANTS="${VARIANTS_U:-lib_variants/v31 lib}" STEPS=4 BENCH_ARGS="--workload zipf_u" bash tools/gpu_ab.sh || exit $?
mkdir -p gpurun_out
[ -f mapreduce_rust_amd/lib_variants/prof/libmrgpu.so ] || exit 0
for w in zipf zipf_u; do
  MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/prof/libmrgpu.so MRG_PROF=1 timeout -k 10 200 python -u bench.py \
    --steps 2 --warmup 1 --quick --workload $w > gpurun_out/phase_$w.log 2>&1 || exit $?
  echo "== $w"; grep -E "phase clocks|step:" gpurun_out/phase_$w.log | tail -3
done
