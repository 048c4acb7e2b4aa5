#!/bin/bash
# r06: where the C3 bucket aggregation's 1.03 ms goes (MRG_AGG_ABLATE: 1 no table adds, 2 no hash
# either, 4 no tail stream; timing only -- results wrong by design), alternated twice.
mkdir -p gpurun_out/aab
for rep in 1 2; do
  for a in 0 1 2 4; do
    MRG_AGG_ABLATE=$a timeout -k 10 200 python3 -u bench.py --steps 6 --warmup 2 --quick > gpurun_out/aab/t$a.log 2>&1 || exit 1
    echo "agg_ablate=$a $(tail -1 gpurun_out/aab/t$a.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print("agg", j["stages_ms"]["ms_aggregate"], "tail", j["job"]["map_records"])')"
  done
done
