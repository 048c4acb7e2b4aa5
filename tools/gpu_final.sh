#!/bin/bash
# Round-end evidence in one call: parity tests, C3 bench (with CPU baselines), kernel-trace profile,
# PMC mix + traffic passes (tools/gpu_full.sh), then the C5 bench and the one-rank shuffle rehearsal.
set -o pipefail
BENCH_STEPS=${BENCH_STEPS:-10} bash tools/gpu_full.sh || exit $?
timeout -k 10 300 python -u bench.py --workload unique --files-per-gpu 50 --steps 3 --warmup 1 --quick > gpurun_out/bench_c5.log 2>&1 || exit $?
echo "c5: $(tail -1 gpurun_out/bench_c5.log | cut -c1-200)"
timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --quick --shuffle-1 > gpurun_out/bench_shuffle1.log 2>&1 || exit $?
echo "shuffle-1: $(tail -1 gpurun_out/bench_shuffle1.log | cut -c1-200)"
FILES=50 bash tools/gpu_c5_prof.sh || exit $?
