#!/bin/bash
# A/B bench variants in one process each, interleaved twice: bash tools/ab.sh "ENV=.. ENV2=.." "ENV=.."
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
for v in "$@"; do
  env $v timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 > gpurun_out/ab/out.json 2>>gpurun_out/ab/err.log || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab/out.json')); print('$v', d['roofline']['kernel_ms'], d['value'], d['roofline']['frac'])"
done; done
