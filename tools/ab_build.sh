#!/bin/bash
# Build a variant of libsvo_rt.so with extra compile definitions into build/ab/<name>/ (A/B runs load it
# through SVO_RT_LIB, raytracingtest_amd/_lib.py), e.g.
#   bash tools/ab_build.sh seg7 -DSVO_SEG_WAVES_PER_EU=1
set -e
name=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/build/ab/$name"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
    -Xarch_device -fno-slp-vectorize -Wno-unused-value -Wno-unused-result "$@" \
    -I"$ROOT/include" -I"$ROOT/raytracingtest_amd/csrc" -o "$ROOT/build/ab/$name/libsvo_rt.so" \
    "$ROOT/raytracingtest_amd/csrc/svo_rt.hip" "$ROOT/raytracingtest_amd/csrc/svo_kernel.hip"
echo "$ROOT/build/ab/$name/libsvo_rt.so"
