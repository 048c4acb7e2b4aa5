#!/bin/bash
# r06: k_map pool claims without a document search per claim; chunk of 4 (lib) vs 8 (lib_variants/k8)
# blocks, pool 1/16 vs 1/8 -- pool parity tests on both builds, then C3 / zipf_u / C5 alternated twice.
mkdir -p gpurun_out/st3
for v in lib lib_variants/k8; do
  MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 240 --timeout-method thread -k "block_pool or c1_wc_golden" > gpurun_out/st3/tests.log 2>&1 \
    || { tail -5 gpurun_out/st3/tests.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/st3/tests.log)"
done
arm() {  # name lib d bench-args
  MRG_LIB=$PWD/mapreduce_rust_amd/$2/libmrgpu.so MRG_MAP_STEAL=$3 timeout -k 10 200 python -u bench.py --quick $4 \
    > gpurun_out/st3/run.log 2>&1 || return 1
  echo "$1 $2 d=$3: median map $(grep 'step:' gpurun_out/st3/run.log | sed 's/.*map \([0-9.]*\) ms.*/\1/' | sort -n | awk '{a[NR]=$1} END {print a[int((NR+1)/2)]}')"
}
for w in "C3|--steps 8 --warmup 2" "zipf_u|--workload zipf_u --steps 5 --warmup 2" "C5|--workload unique --files-per-gpu 16 --steps 4 --warmup 1"; do
  name=${w%%|*}; args=${w#*|}
  for rep in 1 2; do
    for c in "lib 16" "lib 8" "lib_variants/k8 16" "lib_variants/k8 8"; do
      set -- $c
      arm "$name" $1 $2 "$args" || exit 1
    done
  done
done
