mkdir -p gpurun_out
for cap in 1024 2048 4096; do
  timeout -k 10 200 python -u bench.py --files-per-gpu 8 --steps 3 --warmup 1 --quick --lds-cap $cap > gpurun_out/sweep_$cap.log 2>&1 || exit $?
  tail -1 gpurun_out/sweep_$cap.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print($cap, j['value'], j['stages_ms'], j['job']['map_records'])"
done
BENCH_ARGS="--files-per-gpu 4" bash tools/gpu_pmc.sh "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES" "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_LDS" || exit $?
PROF_NAME=r01_v4 bash tools/gpu_prof.sh
