#!/bin/bash
# r06: the exact L2 back as the default -- the wide-path tests (incl. the sampled L2 knob), the C5
# footprint per fresh context, and the one-wave leaf kernel at C5's full size: lib (384 digits, 4 waves
# per SIMD) vs lib_variants/lv512 (512 digits, 3 waves), alternated.
mkdir -p gpurun_out/c5g
timeout -k 10 500 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_ranks.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "l2_sampled or c5_slice or wide_map_forced or wide_packed or wide_many or rare_byte or wide_sample_sort or forced_collisions or cold_context or closed_context" \
  > gpurun_out/c5g/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/c5g/tests.log)"
[ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/c5g/tests.log | head -20; exit $rc; }
FILES=50 timeout -k 10 300 python -u tools/c5_footprint.py > gpurun_out/c5g/footprint.log 2>&1 || { tail -5 gpurun_out/c5g/footprint.log; exit 1; }
cat gpurun_out/c5g/footprint.log | grep L2_SAMPLED
VARIANTS="lib lib_variants/lv512 lib lib_variants/lv512 lib lib_variants/lv512" FILES=50 STEPS=3 bash tools/gpu_c5_ab.sh
