#!/bin/bash
# r05: GPU parity tests (stop on a crash / timeout), then map A/Bs alternated in one box session:
# VARIANTS_U on zipf_u (Gutenberg-like Unicode) and VARIANTS_C3 on C3 (tools/gpu_ab.sh).
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -v -x --timeout 200 --timeout-method thread ${TESTS} > gpurun_out/tests.log 2>&1
  rc=$?
  echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/tests.log | tail -3; grep "^FAILED" gpurun_out/tests.log | head
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "$VARIANTS_U" ]; then
  echo "== zipf_u"; VARIANTS="$VARIANTS_U" STEPS=${STEPS_U:-5} BENCH_ARGS="--workload zipf_u" bash tools/gpu_ab.sh || exit $?
fi
if [ -n "$VARIANTS_C3" ]; then
  echo "== C3"; VARIANTS="$VARIANTS_C3" STEPS=${STEPS_C3:-6} bash tools/gpu_ab.sh || exit $?
fi
exit 0
