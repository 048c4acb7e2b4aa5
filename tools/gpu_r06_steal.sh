#!/bin/bash
# r06: k_map load balance (a pool of the last 1/16 of the blocks, taken by workgroups done with their
# share) -- every GPU test, then A/Bs alternated: lib (pool), lib with MRG_MAP_STEAL=0 (equal shares),
# lib_variants/oldmap (the previous k_map, equal shares) on C3, zipf_u and C5 (16 files).
set -o pipefail
mkdir -p gpurun_out/st
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/st/tests.log 2>&1 || { tail -n 30 gpurun_out/st/tests.log; exit 1; }
tail -n 1 gpurun_out/st/tests.log
arm() {  # name lib steal bench-args
  MRG_LIB=$PWD/mapreduce_rust_amd/$2/libmrgpu.so MRG_MAP_STEAL=$3 timeout -k 10 200 python -u bench.py --quick $4 \
    > gpurun_out/st/run.log 2>&1 || return 1
  echo "$1: $(grep 'step:' gpurun_out/st/run.log | tail -1 | sed 's/.*step: //')  median map $(grep 'step:' gpurun_out/st/run.log | sed 's/.*map \([0-9.]*\) ms.*/\1/' | sort -n | awk '{a[NR]=$1} END {print a[int((NR+1)/2)]}')"
}
for w in "C3|--steps 8 --warmup 2" "zipf_u|--workload zipf_u --steps 5 --warmup 2" "C5|--workload unique --files-per-gpu 16 --steps 4 --warmup 1"; do
  name=${w%%|*}; args=${w#*|}
  for rep in 1 2; do
    arm "$name pool     " lib 1 "$args" || exit 1
    arm "$name shares   " lib 0 "$args" || exit 1
    arm "$name old k_map" lib_variants/oldmap 0 "$args" || exit 1
  done
done
