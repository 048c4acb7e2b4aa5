#!/bin/bash
# r05 v71: uni_class with one LDS read for both fast ranges (EXTRA=-DMRG_MAP_UCB=1 on a k_map.hip with an
# MRG_MAP_UCB branch, not kept in the tree; lib_variants/ucb):
# parity through the variant, then alternated zipf_u and C3 timings against the main build.
set -o pipefail
mkdir -p gpurun_out/v71
MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/ucb/libmrgpu.so timeout -k 10 400 python -u -m pytest -x -q \
  --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > gpurun_out/v71/tests_ucb.log 2>&1 || exit $?
tail -n 1 gpurun_out/v71/tests_ucb.log
BENCH_ARGS="--workload zipf_u" VARIANTS="lib_variants/ucb lib lib_variants/ucb lib lib_variants/ucb lib" \
  bash tools/gpu_ab.sh > gpurun_out/v71/ab_zipf_u.txt || exit $?
VARIANTS="lib_variants/ucb lib lib_variants/ucb lib" bash tools/gpu_ab.sh > gpurun_out/v71/ab_c3.txt || exit $?
cat gpurun_out/v71/ab_zipf_u.txt gpurun_out/v71/ab_c3.txt
