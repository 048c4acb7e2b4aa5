#!/bin/bash
# A/B timing of library variants in one box session: MRG_LIB=<variant>/libmrgpu.so, alternating
# runs, median map / aggregate ms per run.  Usage: VARIANTS="lib_variants/A lib lib_variants/A lib" bash tools/gpu_ab.sh
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-lib_variants/A lib lib_variants/A lib}; do
  MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -k 10 200 python -u bench.py --steps ${STEPS:-8} --warmup 2 \
    --quick ${BENCH_ARGS} > gpurun_out/ab/run.log 2>&1 || exit $?
  python3 - "$v" <<'PY'
import json, re, sys, statistics
lines = open("gpurun_out/ab/run.log").read().splitlines()
m = [float(re.search(r"map ([0-9.]+) ms", l).group(1)) for l in lines if "step: map" in l]
a = [float(re.search(r"agg ([0-9.]+)", l).group(1)) for l in lines if "step: map" in l]
so = [float(re.search(r"sort ([0-9.]+)", l).group(1)) for l in lines if "step: map" in l]
j = json.loads(lines[-1])
print(f"{sys.argv[1]:22s} map median {statistics.median(m):.3f} ms  agg median {statistics.median(a):.3f}  sort {statistics.median(so):.3f}  value {j['value']}  tail {j['job']['map_records']}  tokens {j['job']['tokens']}")
PY
done
