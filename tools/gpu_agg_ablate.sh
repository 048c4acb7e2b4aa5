#!/bin/bash
# Bucket-aggregation ablations (MRG_AGG_ABLATE: 1 = no table adds, 2 = no hash either; timing only,
# results are wrong by design): agg median per level on C3, then SQ counters of each on 1 GiB.
mkdir -p gpurun_out/aab
export TMPDIR=/tmp
for a in 0 1 2; do
  MRG_AGG_ABLATE=$a timeout -k 10 200 python3 -u bench.py --steps 5 --warmup 1 --quick > gpurun_out/aab/t$a.log 2>&1 || exit 1
  echo "agg_ablate=$a $(grep -o '"ms_aggregate": [0-9.]*' gpurun_out/aab/t$a.log)"
done
for a in 0 1; do
  MRG_AGG_ABLATE=$a timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/aab -o p$a --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --quick --files-per-gpu 4 > gpurun_out/aab/p$a.log 2>&1 || exit 1
  python3 tools/pmc_summary.py --dir gpurun_out/aab --glob "p${a}_counter_collection.csv" --only k_bucket_agg | sed "s/^/aab=$a /"
done
