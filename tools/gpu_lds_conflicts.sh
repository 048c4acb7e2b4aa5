#!/bin/bash
# LDS bank conflicts of k_map (C3, FILES x 256 MiB) for the product build and timing variants:
# one rocprofv3 --pmc pass each (SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE, SQ_INSTS_LDS, SQ_WAVE_CYCLES).
mkdir -p gpurun_out/ldsc
export TMPDIR=/tmp
for v in ${VARIANTS:-lib lib_variants/nocount lib_variants/notable}; do
  n=$(basename $v)
  MRG_LIB=$PWD/mapreduce_rust_amd/$v/libmrgpu.so timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    SQ_INSTS_LDS SQ_WAVE_CYCLES -d gpurun_out/ldsc -o $n --output-format csv -- python3 bench.py --files-per-gpu ${FILES:-8} \
    --steps 1 --warmup 1 --quick > gpurun_out/ldsc/$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, os, collections
for f in sorted(glob.glob("gpurun_out/ldsc/**/*counter_collection.csv", recursive=True)):
    t = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "k_map" in r["Kernel_Name"]:
            t[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    if t:
        print(os.path.basename(f), {k: "%.3g" % v for k, v in t.items()},
              "conflict/active %.3f" % (t["SQ_LDS_BANK_CONFLICT"] / max(t["SQ_LDS_IDX_ACTIVE"], 1)))
PY
