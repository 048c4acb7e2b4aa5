#!/bin/bash
# Wide-path GPU tests, then an A/B of library variants on C5 at its stated size (50 x 256 MiB):
#   VARIANTS="lib_variants/H lib" bash tools/gpu_c5_check.sh
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wide or unique or c5" \
  > gpurun_out/ab/wide_tests.log 2>&1 || { tail -30 gpurun_out/ab/wide_tests.log; exit 1; }
tail -2 gpurun_out/ab/wide_tests.log
for v in ${VARIANTS:-lib}; do
  MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -k 10 300 python -u bench.py --workload unique --files-per-gpu ${FILES:-50} \
    --steps ${STEPS:-4} --warmup 1 --quick > gpurun_out/ab/c5.log 2>&1 || exit $?
  echo "$v: $(grep 'step:' gpurun_out/ab/c5.log | tail -1)"
  if [ -n "$DEBUG" ]; then
    MRG_DEBUG=1 MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -k 10 300 python -u bench.py --workload unique \
      --files-per-gpu ${FILES:-50} --steps 2 --warmup 1 --quick > gpurun_out/ab/c5d.log 2>&1 || exit $?
    echo "$v debug: $(grep -E 'wide phases' gpurun_out/ab/c5d.log | tail -1 | tr '\n' ' ')"
  fi
done
