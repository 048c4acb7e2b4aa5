#!/bin/bash
# r06 iteration: the C3 wave sweep (parity of the sweep builds checked by their token counts), the C5
# line-writer variants (parity tests, then A/B), and the C3 line with the cold leg and the end-to-end
# leg (mrg_run_job twice: the second call reuses the first one's device blocks).
mkdir -p gpurun_out
NO_TESTS=1 VARIANTS="lib lib_variants/w12 lib_variants/w8 lib lib_variants/w12 lib_variants/w8" bash tools/gpu_r06_waves.sh > gpurun_out/waves.log 2>&1
rc=$?; cat gpurun_out/waves.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r06_c5w.sh > gpurun_out/c5w.log 2>&1
rc=$?; cat gpurun_out/c5w.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-zipf-u --no-c5 --no-c2 > gpurun_out/c3_e2e.log 2>&1
rc=$?; grep -E "cold job|end-to-end" gpurun_out/c3_e2e.log; exit $rc
