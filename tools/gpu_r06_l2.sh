#!/bin/bash
# r06: sampled L2 leaves (k_wl2) and the one-wave leaf kernel at 4 waves per SIMD -- the wide-path tests
# against the oracle (product, then the leaf variant), the XCD-aware aggregation tests, then A/Bs: C5
# with the sampled vs the exact L2 histogram (MRG_WIDE_L2_EXACT) and the leaf variants; zipf_u with the
# XCD-aware vs the plain sub-range mapping (lib_variants/aggx0).
mkdir -p gpurun_out/ab
WK="l2_sampled or c5_slice or wide_map_forced or wide_packed or wide_many or rare_byte"
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "${TESTK:-$WK or subranges or speculative or closed_context or zipf_unicode or aggregation_overflow}" \
  > gpurun_out/ab/tests_l2.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/ab/tests_l2.log)"
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/ab/tests_l2.log | head -20; exit $rc; }
for v in ${LEAFV:-lv384}; do
  MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/$v/libmrgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py \
    -m gpu -x -q --timeout 300 --timeout-method thread -k "$WK" > gpurun_out/ab/tests_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc: $(tail -1 gpurun_out/ab/tests_$v.log)"
  [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/ab/tests_$v.log | head -20; exit $rc; }
done
for rep in 1 2; do
  for c in "lib 0" "lib 1" "lib_variants/lv384 0" "lib_variants/lv512w4 0"; do
    set -- $c
    MRG_LIB=$PWD/mapreduce_rust_amd/$1/libmrgpu.so MRG_WIDE_L2_EXACT=$2 timeout -k 10 200 python -u bench.py --workload unique \
      --files-per-gpu 16 --steps 4 --warmup 1 --quick > gpurun_out/ab/c5.log 2>&1 || exit $?
    echo "$1 L2_EXACT=$2: $(grep 'step:' gpurun_out/ab/c5.log | tail -1)"
  done
done
VARIANTS="lib lib_variants/aggx0 lib lib_variants/aggx0" STEPS=5 BENCH_ARGS="--workload zipf_u" bash tools/gpu_ab.sh
