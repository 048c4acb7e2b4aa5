#!/bin/bash
# tools/gpu_uni.sh, then an A/B of the C3 (ASCII) map against lib_variants/nouni (the same sources
# built with -DMRG_MAP_NO_UNI: non-ASCII tiles to the exact walker, as in r03).
bash tools/gpu_uni.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VARIANTS="lib_variants/nouni lib lib_variants/nouni lib" STEPS=6 bash tools/gpu_ab.sh || exit $?
exit $rc
