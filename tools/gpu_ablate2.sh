#!/bin/bash
# tools/gpu_ablate.sh on C3 (zipf) and on zipf_u, same ablation set (timing only; ablation build).
for w in zipf zipf_u; do
  echo "== $w"
  BENCH_ARGS="--workload $w" ABLATE_SET="${ABLATE_SET:-0 32 64 4 128}" bash tools/gpu_ablate.sh || exit $?
done
