#!/bin/bash
# r06 item 2: the cold-context paths (tests), then the default bench line with its `cold` legs.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -m gpu -v -x --timeout 300 --timeout-method thread \
  -k "c5_slice or cold_context" > gpurun_out/cold_tests.log 2>&1
rc=$?; echo "cold tests rc=$rc"; grep -E "passed|failed|PASS|FAIL" gpurun_out/cold_tests.log | tail -5
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/default_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/default_bench.log | cut -c1-300; grep "cold job" gpurun_out/default_bench.log
exit $rc
