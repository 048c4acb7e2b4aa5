#!/bin/bash
# r06: cold-path tests + probe + C3 line with the cold and end-to-end legs; C5 L2 / leaf phase clocks.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c5_slice or cold_context" > gpurun_out/cold_tests.log 2>&1 || { tail -30 gpurun_out/cold_tests.log; exit 1; }
tail -1 gpurun_out/cold_tests.log
timeout -k 10 200 python -u tools/cold_probe.py > gpurun_out/cold_probe.log 2>&1 || { tail -20 gpurun_out/cold_probe.log; exit 1; }
grep job gpurun_out/cold_probe.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-zipf-u --no-c5 --no-c2 > gpurun_out/c3_e2e.log 2>&1 || { tail -20 gpurun_out/c3_e2e.log; exit 1; }
grep -E "cold job|end-to-end" gpurun_out/c3_e2e.log
MRG_DEBUG=1 MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/wprof/libmrgpu.so timeout -k 10 200 python -u bench.py --workload unique \
  --files-per-gpu 16 --steps 2 --warmup 1 --quick > gpurun_out/c5_wprof.log 2>&1 || { tail -20 gpurun_out/c5_wprof.log; exit 1; }
grep -E "phase clocks|step:" gpurun_out/c5_wprof.log | tail -6
