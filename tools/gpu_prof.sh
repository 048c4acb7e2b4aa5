#!/bin/bash
# Kernel-trace profile of a short bench run (rocprofv3 --kernel-trace --stats), CSV under gpurun_out/prof.
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o ${PROF_NAME:-run} --output-format csv -- \
    python3 bench.py --steps ${BENCH_STEPS:-5} --warmup 1 --quick ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
rc=$?
echo "prof rc=$rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
