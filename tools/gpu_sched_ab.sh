#!/bin/bash
# r05 v67: k_map built with other AMDGPU scheduler strategies (tools/build_variant.sh with EXTRA =
# -mllvm -amdgpu-sched-strategy=max-ilp | max-memory-clause | iterative-ilp, or
# -amdgpu-set-wave-priority) against the main build: alternated C3, then zipf_u.
set -o pipefail
mkdir -p gpurun_out/v67
VARIANTS="lib_variants/ilp lib_variants/mclause lib_variants/itilp lib_variants/wprio lib lib_variants/ilp lib_variants/mclause lib_variants/itilp lib_variants/wprio lib" \
  bash tools/gpu_ab.sh > gpurun_out/v67/ab_c3.txt || exit $?
cat gpurun_out/v67/ab_c3.txt
BENCH_ARGS="--workload zipf_u" VARIANTS="lib_variants/ilp lib_variants/mclause lib_variants/itilp lib_variants/wprio lib" \
  bash tools/gpu_ab.sh > gpurun_out/v67/ab_zipf_u.txt || exit $?
cat gpurun_out/v67/ab_zipf_u.txt
