#!/bin/bash
# r06: k_map workgroups beyond one per CU (MRG_TEST_MAP_GRID) against the end-of-launch imbalance
# (workgroup end times: median 7.30, max 7.58 ms at 10 GiB, tools/gpu_r06_phase.sh) -- C3 and zipf_u,
# alternated; correctness of the C3 full-size job at the best setting.
mkdir -p gpurun_out/grid
for rep in 1 2; do
  for g in 256 512 384 768; do
    MRG_TEST_MAP_GRID=$g timeout -k 10 200 python -u bench.py --steps 6 --warmup 2 --quick > gpurun_out/grid/c3.log 2>&1 || exit $?
    echo "C3 grid=$g: $(grep 'step:' gpurun_out/grid/c3.log | tail -1 | sed 's/.*step: //')  $(tail -1 gpurun_out/grid/c3.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("value", j["value"], "kmap", j["roofline"]["kernel_ms_median"], "agg", j["stages_ms"]["ms_aggregate"], "tail", j["job"]["map_records"])')"
  done
done
for g in 256 512; do
  MRG_TEST_MAP_GRID=$g timeout -k 10 200 python -u bench.py --workload zipf_u --steps 5 --warmup 2 --quick > gpurun_out/grid/zu.log 2>&1 || exit $?
  echo "zipf_u grid=$g: $(grep 'step:' gpurun_out/grid/zu.log | tail -1 | sed 's/.*step: //')"
done
