#!/bin/bash
# r06: sampled L2, leaf target x region capacity (MRG_TEST_LEAF_TARGET, MRG_TEST_L2_CAP), C5 16 x 256 MiB,
# alternated twice.
mkdir -p gpurun_out/l2e
for rep in 1 2; do
  for c in "288 8,64" "272 8,64" "272 6,64" "256 6,64" "240 6,64"; do
    set -- $c
    MRG_TEST_LEAF_TARGET=$1 MRG_TEST_L2_CAP=$2 timeout -k 10 200 python -u bench.py --workload unique \
      --files-per-gpu 16 --steps 5 --warmup 1 --quick > gpurun_out/l2e/c5.log 2>&1 || exit $?
    echo "target=$1 cap=$2: $(grep 'step:' gpurun_out/l2e/c5.log | tail -1)"
  done
done
