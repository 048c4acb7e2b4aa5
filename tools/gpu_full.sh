#!/bin/bash
# One GPU call: parity tests + bench (C3) + kernel-trace stats + PMC traffic passes.
# Each GPU step has its own time limit; any failing step ends the script.
set -o pipefail
bash tools/gpu_check.sh || exit $?
PROF_NAME=${PROF_NAME:-run} bash tools/gpu_prof.sh || exit $?
bash tools/gpu_counters.sh || exit $?
echo "all done"
