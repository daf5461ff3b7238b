#!/bin/bash
# Latency-form A/B: tools/lat_ab.py (whole frame, strong-split bands N = 2/4/8, the lone heaviest
# tile row; lean / latency / automatic forms, hit records compared between the forms) with each
# library built by tools/ab_lib.sh, two interleaved rounds.
#   bash tools/ab_latform.sh NAME...      [AB_CAMERA=overview]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
for rep in 1 2; do
  for name in "$@"; do
    echo "== $name (round $rep)"
    SVO_RT_LIB="$ROOT/build/ab/libsvo_rt_$name.so" timeout -k 10 300 python tools/lat_ab.py --reps 30 \
      ${AB_CAMERA:+--camera $AB_CAMERA} 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
