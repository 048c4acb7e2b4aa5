#!/bin/bash
# r05 v68: k_wide.hip built with other AMDGPU scheduler strategies against the main build, C5 alternated.
set -o pipefail
mkdir -p gpurun_out/v68
STEPS=3 BENCH_ARGS="--workload unique --files-per-gpu 50" \
  VARIANTS="lib_variants/wilp lib_variants/wmclause lib_variants/witilp lib_variants/wwprio lib lib_variants/wilp lib_variants/wmclause lib_variants/witilp lib_variants/wwprio lib" \
  bash tools/gpu_ab.sh > gpurun_out/v68/ab_c5.txt || exit $?
cat gpurun_out/v68/ab_c5.txt
