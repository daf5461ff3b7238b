#!/bin/bash
# A/B bench variants (one process each, interleaved twice) with the CPU-oracle
# parity check of the bench frame: bash tools/ab_parity.sh "ENV=.." "ENV=.."
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --steps 40 --warmup 10 --cpu-seconds ${CPU_S:-0.5} > gpurun_out/ab/out.json 2>>gpurun_out/ab/err.log || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab/out.json')); c=d['cpu_baseline'] or {}; print('$v', d['roofline']['kernel_ms'], d['value'], d['roofline']['frac'], 'mismatch', c.get('parity_rays_mismatched'), 'of', c.get('parity_rays_checked'))"
done; done
