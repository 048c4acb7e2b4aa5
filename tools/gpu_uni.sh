#!/bin/bash
# Parity tests (stop at the first failure), then short --quick benches of C3 (ASCII) and zipf_u
# (Gutenberg-like Unicode): k_map and step times of both.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${TESTS} > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for w in zipf zipf_u; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --quick > gpurun_out/bench_$w.log 2>&1 || exit $?
  grep "step:" gpurun_out/bench_$w.log | tail -2
  tail -1 gpurun_out/bench_$w.log | cut -c1-300
done
