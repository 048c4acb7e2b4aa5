#!/bin/bash
# r05 round-end evidence in one call: the wide-path tests and a C5 A/B against lib_variants/prev,
# then gpu_full.sh (all GPU tests, the default bench line, kernel-trace stats, PMC mix + traffic),
# the C5 kernel trace and the C5 per-kernel traffic.  Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_scale.py tests/test_gpu_ranks.py -k "wide or c5 or leaf or pack or collision" > gpurun_out/wide_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/wide_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -f mapreduce_rust_amd/lib_variants/prev/libmrgpu.so ]; then
  STEPS=3 BENCH_ARGS="--workload unique --files-per-gpu 50" VARIANTS="lib_variants/prev lib lib_variants/prev lib" \
    bash tools/gpu_ab.sh > gpurun_out/c5_ab.txt 2>&1 || exit $?
  cat gpurun_out/c5_ab.txt
fi
BENCH_STEPS=${BENCH_STEPS:-10} bash tools/gpu_full.sh || exit $?
FILES=50 bash tools/gpu_c5_prof.sh || exit $?
FILES=16 bash tools/gpu_c5_traffic.sh || exit $?
echo "final done"
