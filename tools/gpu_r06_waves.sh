#!/bin/bash
# r06 item 1(a): k_map occupancy sweep -- the product build (16 waves per workgroup = 4 waves/SIMD)
# against MRG_MAP_WAVES 12 (3/SIMD) and 8 (2/SIMD) builds (tools/build_variant.sh), alternated on
# C3 in one box session.  A 20-wave workgroup cannot exist (1024 threads per workgroup at most).
# NO_TESTS=1 skips the GPU test run first.
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -v -x --timeout 200 --timeout-method thread ${TESTS} > gpurun_out/tests.log 2>&1
  rc=$?
  echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/tests.log | tail -3; grep "^FAILED" gpurun_out/tests.log | head
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
echo "== C3 wave sweep"
VARIANTS="${VARIANTS:-lib lib_variants/w12 lib_variants/w8 lib lib_variants/w12 lib_variants/w8}" STEPS=${STEPS:-6} bash tools/gpu_ab.sh
