#!/bin/bash
# r06: the sampled L2's leaf target and region capacity (MRG_TEST_LEAF_TARGET, MRG_TEST_L2_CAP) against
# the exact histogram, C5 16 x 256 MiB, alternated twice.
mkdir -p gpurun_out/l2c
for rep in 1 2; do
  for c in "1 320 8,64" "0 288 8,64" "0 288 5,64" "0 272 5,64" "0 304 5,64"; do
    set -- $c
    MRG_WIDE_L2_EXACT=$1 MRG_TEST_LEAF_TARGET=$2 MRG_TEST_L2_CAP=$3 timeout -k 10 200 python -u bench.py --workload unique \
      --files-per-gpu 16 --steps 4 --warmup 1 --quick > gpurun_out/l2c/c5.log 2>&1 || exit $?
    echo "L2_EXACT=$1 target=$2 cap=$3: $(grep 'step:' gpurun_out/l2c/c5.log | tail -1)"
  done
done
