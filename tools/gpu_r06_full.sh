#!/bin/bash
# r06: every GPU test on the product library, then C5 lib vs lib_variants/lv384 (one-wave leaves at 384
# digits, 4 waves per SIMD), alternated, 16 x 256 MiB.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/tests_full.log 2>&1 || { tail -n 30 gpurun_out/tests_full.log; exit 1; }
tail -n 1 gpurun_out/tests_full.log
VARIANTS="${VARIANTS:-lib lib_variants/lv384 lib lib_variants/lv384 lib lib_variants/lv384}" STEPS=5 bash tools/gpu_c5_ab.sh
