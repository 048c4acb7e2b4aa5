#!/bin/bash
# Build a variant of libmrgpu.so with a modified k_map.hip: tools/build_variant.sh NAME FILE.hip
# -> mapreduce_rust_amd/lib_variants/NAME/libmrgpu.so (other objects from the main build).
set -e
name=$1; src=$2
d=/tmp/var_$name; rm -rf $d; mkdir -p $d
cp mapreduce_rust_amd/csrc/*.h mapreduce_rust_amd/csrc/*.inc $d/
cp $src $d/k_map.hip
(cd $d && /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I/root/repo/include -w ${EXTRA} -c k_map.hip -o k_map.hip.o)
mkdir -p mapreduce_rust_amd/lib_variants/$name
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o mapreduce_rust_amd/lib_variants/$name/libmrgpu.so $d/k_map.hip.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib \
  $(ls mapreduce_rust_amd/lib/obj/*.o | grep -v k_map)
echo built $name
