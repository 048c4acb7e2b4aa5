#!/bin/bash
# r06: the k_map pool's size (MRG_MAP_STEAL = d: a pool of 1/d of the blocks; 0 = none), C3 and zipf_u
# alternated twice; then phase clocks / workgroup end times with the default pool.
mkdir -p gpurun_out/st2
arm() {  # name steal bench-args
  MRG_MAP_STEAL=$2 timeout -k 10 200 python -u bench.py --quick $3 > gpurun_out/st2/run.log 2>&1 || return 1
  echo "$1 d=$2: median map $(grep 'step:' gpurun_out/st2/run.log | sed 's/.*map \([0-9.]*\) ms.*/\1/' | sort -n | awk '{a[NR]=$1} END {print a[int((NR+1)/2)]}')  $(grep 'step:' gpurun_out/st2/run.log | tail -1 | sed 's/.*step: //')"
}
for w in "C3|--steps 8 --warmup 2" "zipf_u|--workload zipf_u --steps 5 --warmup 2"; do
  name=${w%%|*}; args=${w#*|}
  for rep in 1 2; do
    for d in 16 8 32 4 0; do arm "$name" $d "$args" || exit 1; done
  done
done
for w in zipf zipf_u; do
  MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/prof/libmrgpu.so MRG_PROF=1 timeout -k 10 200 python -u bench.py --workload $w \
    --steps 2 --warmup 1 --quick > gpurun_out/st2/ph_$w.log 2>&1 || exit 1
  echo "== $w"; grep -E "phase clocks|map workgroups" gpurun_out/st2/ph_$w.log | tail -2
done
