#!/bin/bash
# r06: a job's small setup writes batched (one copy + one k_stage_scatter instead of a copy or memset
# each) -- every GPU test, then C3 (and C2 latency inside the default line's legs) alternated:
# lib vs lib_variants/nostage.
set -o pipefail
mkdir -p gpurun_out/sg
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/sg/tests.log 2>&1 || { tail -n 30 gpurun_out/sg/tests.log; exit 1; }
tail -n 1 gpurun_out/sg/tests.log
for rep in 1 2 3; do
  for v in lib lib_variants/nostage; do
    MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -k 10 200 python -u bench.py --quick --steps 10 --warmup 2 \
      > gpurun_out/sg/run.log 2>&1 || exit 1
    echo "$v: $(tail -1 gpurun_out/sg/run.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("ms_per_step", j["ms_per_step"], "value", j["value"], "kmap", j["roofline"]["kernel_ms_median"])')"
  done
done
