#!/bin/bash
# End-to-end leg A/B: chunks DMA'd from registered page-cache mappings (default) vs pread into pinned
# buffers (MRG_READ_MMAP=0), alternating, C3 (40 x 256 MiB files).
mkdir -p gpurun_out/e2e
for v in ${E2E_SET:-1 0 1 0}; do
  MRG_READ_MMAP=$v timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-zipf-u --no-c5 --no-c2 \
    > gpurun_out/e2e/run_$v.log 2>&1 || exit $?
  echo "MRG_READ_MMAP=$v: $(grep 'end-to-end:' gpurun_out/e2e/run_$v.log | tail -1)"
done
