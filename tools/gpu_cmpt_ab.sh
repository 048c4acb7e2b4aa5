#!/bin/bash
# r05 v63/v64: compacted codepoint decode variants (built with tools/build_variant.sh, EXTRA=-DMRG_MAP_CMPT=1:
# lib_variants/cmpt, and cmpt2 = cmpt + the edge codepoints folded in) -- parity tests through the
# variant, then alternated zipf_u and C3 timings against the main build (v63 ran cmpt alone).
set -o pipefail
mkdir -p gpurun_out/v64
MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/cmpt2/libmrgpu.so timeout -k 10 400 python -u -m pytest -x -q \
  --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  "tests/test_gpu_scale.py::test_zipf_unicode_256mib_vs_oracle" > gpurun_out/v64/tests_cmpt.log 2>&1 || exit $?
tail -2 gpurun_out/v64/tests_cmpt.log
BENCH_ARGS="--workload zipf_u" VARIANTS="lib_variants/cmpt2 lib_variants/cmpt lib lib_variants/cmpt2 lib_variants/cmpt lib lib_variants/cmpt2 lib_variants/cmpt lib" \
  bash tools/gpu_ab.sh > gpurun_out/v64/ab_zipf_u.txt || exit $?
VARIANTS="lib_variants/cmpt2 lib lib_variants/cmpt2 lib" bash tools/gpu_ab.sh > gpurun_out/v64/ab_c3.txt || exit $?
cat gpurun_out/v64/ab_zipf_u.txt gpurun_out/v64/ab_c3.txt
