#!/bin/bash
# C5: leaf target (MRG_TEST_LEAF_TARGET) A/B on the product build, one bench per setting, alternated.
mkdir -p gpurun_out/ab
for t in ${TARGETS:-256 232 288 256 232 288}; do
  MRG_TEST_LEAF_TARGET=$t timeout -k 10 200 python3 -u bench.py --workload unique --files-per-gpu 50 --steps 5 --warmup 1 \
    --quick > gpurun_out/ab/run.log 2>&1 || exit $?
  echo "target $t $(grep '^{' gpurun_out/ab/run.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stages_ms'])")"
done
