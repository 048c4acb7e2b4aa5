#!/bin/bash
# tools/gpu_uni.sh, then an A/B of the C3 (ASCII) map against lib_variants/base.
bash tools/gpu_uni.sh || exit $?
VARIANTS="lib_variants/base lib lib_variants/base lib" bash tools/gpu_ab.sh || exit $?
