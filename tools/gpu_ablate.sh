#!/bin/bash
# Perf ablations of the map kernel (MRG_ABLATE; results are wrong by design, timing only).
# k_map's ablation knobs exist only in the ablation build:
#   EXTRA=-DMRG_MAP_ABLATION bash tools/build_variant.sh ablation mapreduce_rust_amd/csrc/k_map.hip
export MRG_LIB=${MRG_LIB:-$PWD/mapreduce_rust_amd/lib_variants/ablation/libmrgpu.so}
mkdir -p gpurun_out/ablate
for ab in ${ABLATE_SET:-0 1 2 3 4}; do
  MRG_ABLATE=$ab timeout -k 10 200 python -u bench.py --files-per-gpu ${FILES:-8} --steps 3 --warmup 1 --quick ${BENCH_ARGS} > gpurun_out/ablate/ab$ab.log 2>&1 || exit $?
  tail -1 gpurun_out/ablate/ab$ab.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('ablate', $ab, 'map_ms', j['stages_ms']['ms_map'], 'job GB/s', j['value'], 'tail', j['job']['map_records'])"
done
