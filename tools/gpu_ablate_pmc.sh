#!/bin/bash
# Per-phase instruction counts of k_map: one PMC pass per ablation level (MRG_ABLATE) on 1 GiB of C3,
# then the map time of each level on the full C3 input.  ABLS="32 64 4 0" by default.
# k_map's ablation knobs exist only in the ablation build:
#   EXTRA=-DMRG_MAP_ABLATION bash tools/build_variant.sh ablation mapreduce_rust_amd/csrc/k_map.hip
export MRG_LIB=${MRG_LIB:-$PWD/mapreduce_rust_amd/lib_variants/ablation/libmrgpu.so}
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
CTRS=${CTRS:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}
for a in ${ABLS:-32 64 4 0}; do
  MRG_ABLATE=$a timeout -s KILL 120 rocprofv3 --pmc $CTRS -d gpurun_out/abl -o abl$a --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --quick --files-per-gpu 4 > gpurun_out/abl/abl$a.log 2>&1 || exit $?
  python3 tools/pmc_summary.py --dir gpurun_out/abl --glob "abl${a}_counter_collection.csv" --only k_map | sed "s/^/abl=$a /"
done
for a in ${ABLS:-32 64 4 0}; do
  MRG_ABLATE=$a timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 1 --quick > gpurun_out/abl/t$a.log 2>&1 || exit $?
  echo "abl=$a $(grep -o 'kernel_ms_median": [0-9.]*' gpurun_out/abl/t$a.log)"
done
