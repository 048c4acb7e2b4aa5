#!/bin/bash
# C5 wide path: L2 / leaf phase clocks (diagnostic build) and HBM traffic per kernel (two PMC passes:
# FETCH_SIZE, WRITE_SIZE) over a short near-unique-key bench (FILES x 256 MiB).
mkdir -p gpurun_out/c5pmc
export TMPDIR=/tmp
if [ -f mapreduce_rust_amd/lib_variants/wprof/libmrgpu.so ]; then
  MRG_DEBUG=1 MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/wprof/libmrgpu.so timeout -k 10 300 python3 -u bench.py \
    --workload unique --files-per-gpu 50 --steps 1 --warmup 1 --quick > gpurun_out/c5_wprof.log 2>&1 || exit $?
  grep -E "L2 phase|one-wave|leaf phase|passed to" gpurun_out/c5_wprof.log | tail -5
fi
ARGS="--workload unique --files-per-gpu ${FILES:-16} --steps 1 --warmup 1 --quick"
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/c5pmc -o pass$i --output-format csv -- python3 bench.py $ARGS > gpurun_out/c5pmc/pass$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py --dir gpurun_out/c5pmc > gpurun_out/c5pmc/summary.txt 2>&1; head -40 gpurun_out/c5pmc/summary.txt
