#!/bin/bash
# A/B bench variants (svo_config fields, include/svo_rt.h) in one process each, interleaved twice:
#   bash tools/ab.sh "beam=0 seg_cap=256" "default"
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
for v in "$@"; do
  sets=()
  for kv in $v; do [ "$kv" = default ] || sets+=(--set "$kv"); done
  timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-extras "${sets[@]}" > gpurun_out/ab/out.json 2>>gpurun_out/ab/err.log || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab/out.json')); print('$v', d['roofline']['kernel_ms'], d['value'], d['roofline']['frac'])"
done; done
