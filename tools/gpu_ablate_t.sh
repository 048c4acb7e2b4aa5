for ab in 0 128 256 3 1 4; do
  MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/T/libmrgpu.so MRG_ABLATE=$ab timeout -k 10 200 python -u bench.py --files-per-gpu 8 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/abl.log 2>&1 || exit $?
  python3 -c "
import re,statistics
m=[float(re.search(r'map ([0-9.]+) ms',l).group(1)) for l in open('gpurun_out/abl.log') if 'step: map' in l]
print('ablate $ab map median', statistics.median(m))"
done
