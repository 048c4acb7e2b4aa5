#!/bin/bash
# One-sweep vs three-kernel radix passes (MRG_NO_ONESWEEP) on C3, parity tests with one-sweep.
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?; tail -1 gpurun_out/tests.log; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/ab
for v in 1 0 1 0; do
  if [ $v = 1 ]; then export MRG_NO_ONESWEEP=1; else unset MRG_NO_ONESWEEP; fi
  timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/run.log 2>&1 || exit $?
  echo "no_onesweep=$v $(grep step: gpurun_out/ab/run.log | tail -1)"
done
