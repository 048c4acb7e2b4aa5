# k_map's ablation knobs exist only in the ablation build:
#   EXTRA=-DMRG_MAP_ABLATION bash tools/build_variant.sh ablation mapreduce_rust_amd/csrc/k_map.hip
export MRG_LIB=${MRG_LIB:-$PWD/mapreduce_rust_amd/lib_variants/ablation/libmrgpu.so}
set -e
for ab in 0 1 2 16 32 64; do
  MRG_ABLATE=$ab timeout -k 10 120 python bench.py --steps 5 --warmup 2 --quick > gpurun_out/abl_$ab.log 2>&1
done
MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/mprof/libmrgpu.so MRG_PROF=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --quick > gpurun_out/abl_prof.log 2>&1
