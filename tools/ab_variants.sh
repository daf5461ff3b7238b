#!/bin/bash
# Kernel-source A/B: libraries built by `tools/ab_lib.sh build NAME -D...`, each measured in its own
# processes, two interleaved rounds: C3 flyover and Main-pose frames (bench.py --no-extras, kernel
# time) and the lone heaviest tile row with the lean loop (tools/lone_row.py, SVO_LAT=0).
#   bash tools/ab_variants.sh NAME...
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for name in "$@"; do
    lib="$ROOT/build/ab/libsvo_rt_$name.so"
    line="$name"
    for cam in ${AB_CAMS:-flyover main}; do
      SVO_RT_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 20 --cpu-seconds 0 --no-extras --camera $cam \
        > gpurun_out/ab/out.json 2>>gpurun_out/ab/err.log || exit $?
      line="$line $cam $(python3 -c "import json; d=json.load(open('gpurun_out/ab/out.json')); print(d['roofline']['kernel_ms'])")"
    done
    r=$(SVO_LAT=0 SVO_RT_LIB=$lib timeout -k 10 200 python tools/lone_row.py --reps 30 2>>gpurun_out/ab/err.log) || exit $?
    echo "$line | $r"
  done
done
