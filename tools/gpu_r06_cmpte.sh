#!/bin/bash
# r06: edge codepoints in k_map's compacted decode (MRG_MAP_CMPTE 0 / 1 = product / 2) -- the Unicode and
# UTF-8 parity tests on the product and on cmpte2, then k_map A/Bs alternated: zipf_u and C3.
mkdir -p gpurun_out/ab
K="unicode or utf or tile or invalid or zipf or density or edge or kat or short"
for v in lib lib_variants/cmpte2; do
  MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py \
    -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/ab/tests_$(basename $v).log 2>&1
  rc=$?; echo "$v tests rc=$rc: $(tail -1 gpurun_out/ab/tests_$(basename $v).log)"
  [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/ab/tests_$(basename $v).log | head -20; exit $rc; }
done
echo "== zipf_u"
VARIANTS="lib_variants/cmpte0 lib lib_variants/cmpte2 lib_variants/cmpte0 lib lib_variants/cmpte2" STEPS=5 BENCH_ARGS="--workload zipf_u" bash tools/gpu_ab.sh || exit $?
echo "== C3"
VARIANTS="lib_variants/cmpte0 lib lib_variants/cmpte0 lib" STEPS=6 bash tools/gpu_ab.sh || exit $?
