#!/bin/bash
# Instruction-cache PMC of the map kernel on 2 GiB of C3 and zipf_u (one rocprofv3 pass each).
mkdir -p gpurun_out
for w in zipf zipf_u; do
  rm -rf gpurun_out/pmc
  BENCH_ARGS="--files-per-gpu 8 --workload $w" bash tools/gpu_pmc.sh \
    "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU" || exit $?
  mkdir -p gpurun_out/icache_$w && cp -r gpurun_out/pmc/* gpurun_out/icache_$w/
  python3 - "$w" <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob("gpurun_out/pmc/**/*counter_collection*.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
tot = collections.defaultdict(float); n = collections.Counter()
for r in rows:
    if "k_map" not in r.get("Kernel_Name", ""): continue
    tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
print(sys.argv[1], {k: "%.3e" % v for k, v in sorted(tot.items())}, "dispatch-rows", dict(n))
PY
done
