#!/bin/bash
# r06: where the sampled L2 loses -- kernel traces of C5 (16 x 256 MiB) with the sampled and the exact L2
# histogram, then the sampled form at lower leaf targets (the sampled leaves vary more: fewer past the
# one-wave capacity) against the exact one.
mkdir -p gpurun_out/l2b && cd /tmp && export TMPDIR=/tmp
for e in 0 1; do
  MRG_WIDE_L2_EXACT=$e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/l2b/e$e -o run \
    -- python3 $GRAFT_REPO_ROOT/bench.py --workload unique --files-per-gpu 16 --steps 3 --warmup 1 --quick \
    > $GRAFT_REPO_ROOT/gpurun_out/l2b/e$e.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for c in "1 320" "0 320" "0 288" "0 256"; do
    set -- $c
    MRG_WIDE_L2_EXACT=$1 MRG_TEST_LEAF_TARGET=$2 timeout -k 10 200 python -u bench.py --workload unique \
      --files-per-gpu 16 --steps 4 --warmup 1 --quick > gpurun_out/l2b/c5.log 2>&1 || exit $?
    echo "L2_EXACT=$1 target=$2: $(grep 'step:' gpurun_out/l2b/c5.log | tail -1)"
  done
done
