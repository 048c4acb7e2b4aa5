#!/bin/bash
# r06: the sampled L2's leaf target with the 4-wave leaf kernel (MRG_TEST_LEAF_TARGET), C5 16 x 256 MiB,
# alternated twice.
mkdir -p gpurun_out/l2d
for rep in 1 2; do
  for t in 288 256 272 304 320; do
    MRG_TEST_LEAF_TARGET=$t timeout -k 10 200 python -u bench.py --workload unique \
      --files-per-gpu 16 --steps 5 --warmup 1 --quick > gpurun_out/l2d/c5.log 2>&1 || exit $?
    echo "target=$t: $(grep 'step:' gpurun_out/l2d/c5.log | tail -1)"
  done
done
