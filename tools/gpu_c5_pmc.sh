#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each) over a short C5 bench (near-unique keys, FILES x 256 MiB).
mkdir -p gpurun_out/c5pmc
export TMPDIR=/tmp
ARGS="--workload unique --files-per-gpu ${FILES:-8} --steps 1 --warmup 1 --quick"
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/c5pmc -o pass$i --output-format csv -- python3 bench.py $ARGS > gpurun_out/c5pmc/pass$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
