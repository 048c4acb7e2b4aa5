#!/bin/bash
# Quick GPU iteration: parity tests (stop at first failure) then a short C3 bench.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -15 gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --quick ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -4 gpurun_out/bench.log
exit $rc2
