#!/bin/bash
# Parity tests (up to 5 failures reported), then short --quick benches of C3 (ASCII), zipf_u
# (Gutenberg-like Unicode) and C5.  The benches run after ordinary test failures (pytest rc 1) but
# not after a crash, abort or timeout.
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 200 --timeout-method thread ${TESTS} > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/tests.log | tail -3; grep "^FAILED" gpurun_out/tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for w in zipf zipf_u; do
  timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --quick > gpurun_out/bench_$w.log 2>&1 || exit $?
  grep "step:" gpurun_out/bench_$w.log | tail -2
  tail -1 gpurun_out/bench_$w.log | cut -c1-400
done
timeout -k 10 300 python -u bench.py --workload unique --files-per-gpu 50 --steps 3 --warmup 1 --quick > gpurun_out/bench_c5.log 2>&1 || exit $?
grep "step:" gpurun_out/bench_c5.log | tail -2
exit $rc
