#!/bin/bash
# Quick bench + k_map HBM write traffic (one WRITE_SIZE pass) on C3.
bash tools/gpu_quick.sh || exit $?
rm -rf gpurun_out/pmc
BENCH_ARGS="" bash tools/gpu_pmc.sh "WRITE_SIZE" || exit $?
python3 tools/pmc_summary.py --dir gpurun_out/pmc | head -3
