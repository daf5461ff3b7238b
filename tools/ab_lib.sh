#!/bin/bash
# Compile-flag A/B of libsvo_rt.so.
#   build (CPU):  bash tools/ab_lib.sh build NAME [hipcc flags...]   -> build/ab/libsvo_rt_NAME.so
#   run   (GPU):  [AB_ARGS="--camera overview"] bash tools/ab_lib.sh run NAME...   (two interleaved rounds, one process each)
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" = build ]; then
  name=$2; shift 2
  mkdir -p "$ROOT/build/ab"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math -Xarch_device -fno-slp-vectorize \
    -Wno-unused-value -Wno-unused-result -I"$ROOT/include" -I"$ROOT/raytracingtest_amd/csrc" "$@" \
    -o "$ROOT/build/ab/libsvo_rt_$name.so" "$ROOT/raytracingtest_amd/csrc/svo_rt.hip" "$ROOT/raytracingtest_amd/csrc/svo_kernel.hip"
  exit $?
fi
shift
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for name in "$@"; do
    SVO_RT_LIB="$ROOT/build/ab/libsvo_rt_$name.so" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 $AB_ARGS \
      > gpurun_out/ab/out.json 2>>gpurun_out/ab/err.log || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab/out.json')); print('$name', d['roofline']['kernel_ms'], d['value'], d['roofline']['frac'])"
  done
done
