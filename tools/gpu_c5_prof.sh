#!/bin/bash
# Kernel-trace stats of a short C5 bench (near-unique keys).
mkdir -p gpurun_out/c5p
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5p -o c5 --output-format csv -- \
    python3 bench.py --workload unique --files-per-gpu ${FILES:-40} --steps 3 --warmup 1 --quick > gpurun_out/c5p.log 2>&1 || exit $?
grep "step:" gpurun_out/c5p.log | tail -2
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/c5p/c5_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:16]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d}  {r['Name'][:90]}")
PY
