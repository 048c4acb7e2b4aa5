#!/bin/bash
# A/B of library variants on C5 (near-unique keys, 16 files = 4 GiB to keep the call short).
mkdir -p gpurun_out/ab
for v in ${VARIANTS}; do
  MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -k 10 200 python -u bench.py --workload unique --files-per-gpu ${FILES:-16} \
    --steps ${STEPS:-4} --warmup 1 --quick > gpurun_out/ab/c5.log 2>&1 || exit $?
  echo "$v: $(grep 'step:' gpurun_out/ab/c5.log | tail -1)"
done
