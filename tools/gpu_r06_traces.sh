#!/bin/bash
# r06 closing kernel traces of the final sources: smoke(), the C3 / zipf_u / C5 kernel-trace stats.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 \
  || { tail -n 20 gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
PROF_NAME=c3 bash tools/gpu_prof.sh || exit $?
mkdir -p gpurun_out/zp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/zp -o zipf_u --output-format csv -- \
    python3 bench.py --workload zipf_u --steps 5 --warmup 1 --quick > gpurun_out/zp.log 2>&1 || exit $?
FILES=50 bash tools/gpu_c5_prof.sh || exit $?
find gpurun_out/prof gpurun_out/zp gpurun_out/c5p -name "*kernel_stats.csv"
echo "traces done"
