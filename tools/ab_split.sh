#!/bin/bash
# A/B of the heavy-tile split (SVO_HEAVY_SPLIT=K), one process per setting, two
# interleaved rounds: C3 kernel time + step rate, and the bench's CPU-oracle parity
# sample of the same frames (parity_rays_mismatched must stay 0).
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for k in "$@"; do
    SVO_HEAVY_SPLIT=$k timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 1 --no-extras $AB_ARGS \
      > gpurun_out/ab/split.json 2>>gpurun_out/ab/err.log || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab/split.json')); c=d['cpu_baseline']; print('split', $k, 'kernel_ms', d['roofline']['kernel_ms'], 'Mrays/s', d['value'], 'parity', c['parity_rays_checked'], c['parity_rays_mismatched'])"
  done
done
