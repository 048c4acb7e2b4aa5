#!/bin/bash
# Instruction mix / stall split of the map kernel on 2 GiB (two PMC passes) -> gpurun_out/mix_now.txt
rm -rf gpurun_out/pmc
BENCH_ARGS="--files-per-gpu 8" bash tools/gpu_pmc.sh \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT" || exit $?
python3 tools/pmc_summary.py --dir gpurun_out/pmc > gpurun_out/mix_now.txt
head -24 gpurun_out/mix_now.txt
