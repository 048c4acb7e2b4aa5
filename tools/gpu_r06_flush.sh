#!/bin/bash
# r06: k_map's end-of-launch flush with LDS-only barriers (the tail stores drain behind it) -- parity
# tests, then C3 / zipf_u / C5 alternated (lib vs lib_variants/syncflush = the __syncthreads flush),
# then phase clocks / workgroup ends with the prof build.
mkdir -p gpurun_out/fl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 240 --timeout-method thread \
  -k "block_pool or c1_wc_golden or invalid or density or unicode or c3_full or c5_slice or wide_map_forced or long or tile" \
  > gpurun_out/fl/tests.log 2>&1 || { tail -5 gpurun_out/fl/tests.log; grep -E "^E |FAILED" gpurun_out/fl/tests.log | head; exit 1; }
tail -1 gpurun_out/fl/tests.log
arm() {  # name lib bench-args
  MRG_LIB=$PWD/mapreduce_rust_amd/$2/libmrgpu.so timeout -k 10 200 python -u bench.py --quick $3 > gpurun_out/fl/run.log 2>&1 || return 1
  echo "$1 $2: median map $(grep 'step:' gpurun_out/fl/run.log | sed 's/.*map \([0-9.]*\) ms.*/\1/' | sort -n | awk '{a[NR]=$1} END {print a[int((NR+1)/2)]}')  $(grep 'step:' gpurun_out/fl/run.log | tail -1 | sed 's/.*step: //')"
}
for w in "C3|--steps 8 --warmup 2" "zipf_u|--workload zipf_u --steps 5 --warmup 2" "C5|--workload unique --files-per-gpu 16 --steps 4 --warmup 1"; do
  name=${w%%|*}; args=${w#*|}
  for rep in 1 2 3; do
    arm "$name" lib "$args" || exit 1
    arm "$name" lib_variants/syncflush "$args" || exit 1
  done
done
for w in zipf zipf_u; do
  MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/prof/libmrgpu.so MRG_PROF=1 timeout -k 10 200 python -u bench.py \
    --workload $w --steps 2 --warmup 1 --quick > gpurun_out/fl/ph_$w.log 2>&1 || exit 1
  echo "== $w"; grep -E "phase clocks|map workgroups" gpurun_out/fl/ph_$w.log | tail -2
done
