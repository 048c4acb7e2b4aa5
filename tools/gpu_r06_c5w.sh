#!/bin/bash
# r06: C5 line-writer variants -- parity of each against the oracle (wide-path tests), then an A/B
# alternated on C5 (16 x 256 MiB).  VARIANTS: library dirs under mapreduce_rust_amd/ ("lib" = product).
mkdir -p gpurun_out/ab
for v in ${TESTV:-lib lib_variants/wwave}; do
  MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "${TESTK:-c5_slice or wide_map_forced or wide_packed or wide_many}" \
    > gpurun_out/ab/tests_$(basename $v).log 2>&1
  rc=$?; echo "$v tests rc=$rc: $(tail -1 gpurun_out/ab/tests_$(basename $v).log)"
  [ $rc -ne 0 ] && exit $rc
done
VARIANTS="${VARIANTS:-lib lib_variants/wst0 lib_variants/wwave lib lib_variants/wst0 lib_variants/wwave}" bash tools/gpu_c5_ab.sh
