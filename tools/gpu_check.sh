#!/bin/bash
# GPU-box check: parity tests, then a short bench.  Stops on a fault/abort/timeout exit status.
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps ${BENCH_STEPS:-3} --warmup 1 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -3 gpurun_out/bench.log
exit $rc2
