#!/bin/bash
# Per-phase wave clocks of the map kernel (MRG_PROF=1) on 2 GiB, plus the unprofiled timing.
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --files-per-gpu ${FILES:-8} --steps 2 --warmup 1 --quick ${BENCH_ARGS} > gpurun_out/phase_ref.log 2>&1 || exit $?
grep "step:" gpurun_out/phase_ref.log | tail -1
MRG_PROF=1 timeout -k 10 200 python -u bench.py --files-per-gpu ${FILES:-8} --steps 2 --warmup 1 --quick ${BENCH_ARGS} > gpurun_out/phase.log 2>&1 || exit $?
grep "phase clocks" gpurun_out/phase.log | tail -2
grep "step:" gpurun_out/phase.log | tail -1
