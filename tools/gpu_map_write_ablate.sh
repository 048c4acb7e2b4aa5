#!/bin/bash
# Where k_map's writes go (C3): WRITE_SIZE / FETCH_SIZE of k_map for the product build and for a
# build whose map appends no tail records (MRG_MAP_ABL_CONST=1: timing/traffic only, wrong output).
mkdir -p gpurun_out/mapw
export TMPDIR=/tmp
for v in ${VARIANTS:-lib lib_variants/notail}; do
  n=$(basename $v)
  for c in WRITE_SIZE FETCH_SIZE; do
    MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -s KILL 150 rocprofv3 --pmc $c -d gpurun_out/mapw -o ${n}_$c \
      --output-format csv -- python3 bench.py --steps 1 --warmup 1 --quick ${BENCH_ARGS} > gpurun_out/mapw/${n}_$c.log 2>&1
    rc=$?
    echo "$n $c rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
python3 - <<'PY'
import csv, glob, os, json
for f in sorted(glob.glob("gpurun_out/mapw/**/*counter_collection.csv", recursive=True)):
    tot = {}
    for r in csv.DictReader(open(f)):
        if "k_map" in r["Kernel_Name"]:
            key = (r["Dispatch_Id"], r["Counter_Name"])
            tot[key] = tot.get(key, 0.0) + float(r["Counter_Value"])
    vals = sorted(tot.items())
    print(os.path.basename(f), [(k[1], round(v / 2**20, 3)) for k, v in vals], "GiB per k_map dispatch (KiB counters / 2^20)")
PY
for v in ${VARIANTS:-lib lib_variants/notail}; do n=$(basename $v); grep '^{' gpurun_out/mapw/${n}_WRITE_SIZE.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', 'map_records', d['job']['map_records'], 'tokens', d['job']['tokens'])"; done
