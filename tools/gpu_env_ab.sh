#!/bin/bash
# A/B timing of environment settings in one box session (alternating runs of the in-tree library):
# ENVS="MRG_MAP_DYN_PCT=0 MRG_MAP_DYN_PCT=10" bash tools/gpu_env_ab.sh  (use , to set several in one)
mkdir -p gpurun_out/ab
for e in ${ENVS}; do
  env ${e//,/ } timeout -k 10 200 python -u bench.py --steps ${STEPS:-8} --warmup 2 \
    --quick ${BENCH_ARGS} > gpurun_out/ab/run.log 2>&1 || exit $?
  python3 - "$e" <<'PY'
import json, re, sys, statistics
lines = open("gpurun_out/ab/run.log").read().splitlines()
m = [float(re.search(r"map ([0-9.]+) ms", l).group(1)) for l in lines if "step: map" in l]
a = [float(re.search(r"agg ([0-9.]+)", l).group(1)) for l in lines if "step: map" in l]
so = [float(re.search(r"sort ([0-9.]+)", l).group(1)) for l in lines if "step: map" in l]
j = json.loads(lines[-1])
print(f"{sys.argv[1]:34s} map median {statistics.median(m):.3f} ms  agg {statistics.median(a):.3f}  sort {statistics.median(so):.3f}  step {j['ms_per_step']}  value {j['value']}  tail {j['job']['map_records']}")
PY
done
