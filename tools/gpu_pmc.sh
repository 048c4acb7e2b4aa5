#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc run each) over a short bench; CSV under gpurun_out/pmc.
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --quick ${BENCH_ARGS}"
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/pmc -o pass$i --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/pass$i.log 2>&1
  rc=$?
  echo "pass $i ($ctrs) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
