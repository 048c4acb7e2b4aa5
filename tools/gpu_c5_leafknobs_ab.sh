mkdir -p gpurun_out/ab
for v in "lib" "lib_variants/vq2" "lib_variants/vq8" "lib T300" "lib" "lib_variants/vq2" "lib_variants/vq8" "lib T300"; do
  set -- $v; lib=$1; envs=""; [ "$2" = "T300" ] && envs="MRG_TEST_LEAF_TARGET=300"
  env $envs MRG_LIB=$PWD/mapreduce_rust_amd/$lib/libmrgpu.so timeout -k 10 200 python3 -u bench.py --workload unique --files-per-gpu 50 --steps 3 --warmup 1 --quick > gpurun_out/ab/run.log 2>&1 || exit $?
  echo "$v $(grep 'step:' gpurun_out/ab/run.log | tail -1)"
done
