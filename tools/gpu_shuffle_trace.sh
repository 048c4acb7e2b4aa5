#!/bin/bash
# Where the one-rank shuffle rehearsal's step time goes: rocprofv3 runtime trace (HIP API + kernels +
# copies) of bench.py --shuffle-1, summarised by tools/api_summary.py.
mkdir -p gpurun_out/sht
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --runtime-trace --stats -d gpurun_out/sht -o sht --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --quick --shuffle-1 ${BENCH_ARGS} > gpurun_out/sht.log 2>&1 || exit $?
grep "step:" gpurun_out/sht.log | tail -2
ls gpurun_out/sht
python3 tools/api_summary.py gpurun_out/sht > gpurun_out/sht_summary.txt 2>&1
head -60 gpurun_out/sht_summary.txt
