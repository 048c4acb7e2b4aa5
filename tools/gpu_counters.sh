#!/bin/bash
# Counter passes for the map kernel: instruction mix / wait split on 1 GiB, then HBM traffic
# (FETCH_SIZE, WRITE_SIZE: one pass each) on the full C3 input so bench.py can report
# roofline.traffic.  Each pass is its own rocprofv3 run under timeout -s KILL.
mkdir -p gpurun_out
rm -rf gpurun_out/pmc gpurun_out/pmc_traffic
BENCH_ARGS="--files-per-gpu 4" bash tools/gpu_pmc.sh \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" || exit $?
mv gpurun_out/pmc gpurun_out/pmc_mix
BENCH_ARGS="" bash tools/gpu_pmc.sh "FETCH_SIZE" "WRITE_SIZE" || exit $?
mv gpurun_out/pmc gpurun_out/pmc_traffic
python3 tools/pmc_summary.py --dir gpurun_out/pmc_mix > gpurun_out/pmc_mix_summary.txt
python3 tools/pmc_summary.py --dir gpurun_out/pmc_traffic --traffic 10737418240 --out gpurun_out/map_traffic.json \
  --stages 10737418240 --stages-out gpurun_out/stage_traffic.json > gpurun_out/pmc_traffic_summary.txt
