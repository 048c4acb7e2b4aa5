# correctness of variant D through the full GPU suite, then A/B
MRG_LIB=$PWD/mapreduce_rust_amd/lib_variants/${V:-D}/libmrgpu.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_D.log 2>&1
rc=$?; tail -2 gpurun_out/tests_D.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="lib_variants/base lib_variants/${V:-D} lib_variants/base lib_variants/${V:-D}" bash tools/gpu_ab.sh
