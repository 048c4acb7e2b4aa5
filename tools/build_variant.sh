#!/bin/bash
# Build a variant of libmrgpu.so with one source replaced:
#   tools/build_variant.sh NAME FILE.hip [TARGET]   (TARGET: the source it replaces, default k_map.hip)
# -> mapreduce_rust_amd/lib_variants/NAME/libmrgpu.so (other objects from the main build).  EXTRA = more flags.
set -e
name=$1; src=$2; tgt=${3:-k_map.hip}
d=/tmp/var_$name; rm -rf $d; mkdir -p $d
cp mapreduce_rust_amd/csrc/*.h mapreduce_rust_amd/csrc/*.inc $d/
cp $src $d/$tgt
(cd $d && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I/root/repo/include -w ${EXTRA} -c $tgt -o $tgt.o)
mkdir -p mapreduce_rust_amd/lib_variants/$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o mapreduce_rust_amd/lib_variants/$name/libmrgpu.so $d/$tgt.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib \
  $(ls mapreduce_rust_amd/lib/obj/*.o | grep -v "/$tgt.o")
echo built $name
