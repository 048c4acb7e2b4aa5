#!/bin/bash
# One iteration on the GPU box: parity tests on the in-tree library, then an A/B of library variants
# (VARIANTS, see gpu_ab.sh).  Any failing step ends the script.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_ab.sh
