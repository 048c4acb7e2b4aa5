#!/bin/bash
# r06 closing evidence of the final sources in one call: every GPU test, the PMC passes that key
# profiles/map_traffic.json + stage_traffic.json to kernel_src_sha, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ \
  > gpurun_out/tests_final.log 2>&1 || { tail -n 30 gpurun_out/tests_final.log; exit 1; }
tail -n 1 gpurun_out/tests_final.log
bash tools/gpu_counters.sh || exit $?
cp gpurun_out/map_traffic.json gpurun_out/stage_traffic.json profiles/  # this box's copy: the bench reads them
timeout -k 10 600 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -n 20 gpurun_out/bench_final.log; exit 1; }
tail -n 1 gpurun_out/bench_final.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('value', j['value'], 'zipf_u', j.get('zipf_u',{}).get('k_map_vs_ascii'), 'c5', j.get('c5',{}).get('value'), 'traffic', j['roofline'].get('traffic'), 'cold', j.get('cold',{}).get('kernels_vs_steady'), 'c5cold', j.get('c5',{}).get('cold',{}).get('kernels_vs_steady'))"
echo "evidence done"
