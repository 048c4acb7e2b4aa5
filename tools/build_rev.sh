#!/bin/bash
# Build libmrgpu.so of a git revision into mapreduce_rust_amd/lib_variants/NAME (for A/B runs against
# the working tree):  tools/build_rev.sh NAME [REV=HEAD]
set -e
name=$1; rev=${2:-HEAD}
d=/tmp/rev_$name; rm -rf $d; mkdir -p $d
git archive $rev include mapreduce_rust_amd/csrc | tar -x -C $d
# entry points newer than the revision, as stubs that fail (A/B runs of older sources only)
if ! grep -q "mrg_gen_text" $d/mapreduce_rust_amd/csrc/mrgpu.cpp; then
  echo 'extern "C" int mrg_gen_text(void *, void *, unsigned long long, unsigned long long, unsigned long long, unsigned, double, unsigned) { return -1; }' >> $d/mapreduce_rust_amd/csrc/mrgpu.cpp
fi
make -s -j8 -C $d/mapreduce_rust_amd/csrc ../lib/libmrgpu.so >/dev/null
mkdir -p mapreduce_rust_amd/lib_variants/$name
cp $d/mapreduce_rust_amd/lib/libmrgpu.so mapreduce_rust_amd/lib_variants/$name/
echo built $name from $(git rev-parse --short $rev)
