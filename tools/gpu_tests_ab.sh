#!/bin/bash
# Parity tests (stop on a crash / timeout), then tools/gpu_ab_phase.sh (VARIANTS_C3, VARIANTS_U).
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread ${TESTS} > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/tests.log | tail -3; grep "^FAILED" gpurun_out/tests.log | head
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_ab_phase.sh
