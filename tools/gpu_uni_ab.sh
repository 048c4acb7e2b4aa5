#!/bin/bash
# tools/gpu_uni.sh (tests + C3 / zipf_u / C5 benches), then A/Bs of the map against
# lib_variants/tile (-DMRG_MAP_BR=0: tile-by-tile rounds, 16 waves) on C3 and on zipf_u.
bash tools/gpu_uni.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VARIANTS="lib_variants/tile lib lib_variants/tile lib" STEPS=6 bash tools/gpu_ab.sh || exit $?
VARIANTS="lib_variants/tile lib" STEPS=4 BENCH_ARGS="--workload zipf_u" bash tools/gpu_ab.sh || exit $?
exit $rc
