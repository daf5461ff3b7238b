#!/bin/bash
# XCD strip-width A/B (libraries from tools/ab_lib.sh build kK -DSVO_STRIP_K=K): kernel times
# (tools/ab_variants.sh), then each variant's bench frame checked against the CPU oracle.
#   bash tools/ab_strips.sh k1 k2 ...
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
bash "$ROOT/tools/ab_variants.sh" "$@" || exit $?
for name in "$@"; do
  SVO_RT_LIB="$ROOT/build/ab/libsvo_rt_$name.so" timeout -k 10 200 python bench.py --steps 50 --warmup 5 --cpu-seconds 2 \
    --no-extras > gpurun_out/ab/par.json 2>>gpurun_out/ab/err.log || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab/par.json')); c=d['cpu_baseline']; print('$name parity', c['parity_rays_mismatched'], 'of', c['parity_rays_checked'])"
done
