#!/bin/bash
# zipf_u (Gutenberg-like Unicode C3 text): rocprofv3 kernel trace of a short bench, then the PMC mix
# passes of tools/gpu_counters.sh on 1 GiB of it.
mkdir -p gpurun_out/uprof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/uprof -o zipf_u --output-format csv -- \
    python3 bench.py --workload zipf_u --steps 5 --warmup 1 --quick > gpurun_out/uprof.log 2>&1 || exit $?
grep "step:" gpurun_out/uprof.log | tail -2
rm -rf gpurun_out/pmc
BENCH_ARGS="--workload zipf_u --files-per-gpu 4" bash tools/gpu_pmc.sh \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" || exit $?
python3 tools/pmc_summary.py --dir gpurun_out/pmc > gpurun_out/zipf_u_pmc_mix_summary.txt
head -20 gpurun_out/zipf_u_pmc_mix_summary.txt
