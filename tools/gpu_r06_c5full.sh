#!/bin/bash
# r06: the sampled L2 at C5's full size (50 x 256 MiB): kernel traces of the sampled and the exact L2
# histogram, then an A/B alternated twice (sampled target 256 / exact 320 / sampled target 320).
mkdir -p gpurun_out/c5f && cd /tmp && export TMPDIR=/tmp
for e in 0 1; do
  MRG_WIDE_L2_EXACT=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/c5f/e$e -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --workload unique --files-per-gpu 50 --steps 3 --warmup 1 --quick \
    > $GRAFT_REPO_ROOT/gpurun_out/c5f/e$e.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for c in "0 256" "1 320" "0 320"; do
    set -- $c
    MRG_WIDE_L2_EXACT=$1 MRG_TEST_LEAF_TARGET=$2 timeout -k 10 300 python -u bench.py --workload unique \
      --files-per-gpu 50 --steps 3 --warmup 1 --quick > gpurun_out/c5f/c5.log 2>&1 || exit $?
    echo "L2_EXACT=$1 target=$2: $(grep 'step:' gpurun_out/c5f/c5.log | tail -1)"
  done
done
