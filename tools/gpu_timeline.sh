#!/bin/bash
# Kernel trace of a short C3 bench run and the timeline of its last step (tools/step_timeline.py).
mkdir -p gpurun_out/tl
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl -o tl --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --quick ${BENCH_ARGS} > gpurun_out/tl.log 2>&1 || exit $?
python3 tools/step_timeline.py gpurun_out/tl/tl_kernel_trace.csv > gpurun_out/timeline.txt
tail -45 gpurun_out/timeline.txt
