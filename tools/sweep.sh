#!/bin/bash
# Kernel-shape sweep on one GPU: prints "<env> kernel_ms value" per variant.
set -o pipefail
mkdir -p gpurun_out/sweep
run() {
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 > gpurun_out/sweep/out.json 2>>gpurun_out/sweep/err.log || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/sweep/out.json')); print('$*', d['roofline']['kernel_ms'], d['value'])"
}
run SVO_KERNEL=tile || exit $?
for r in 0 16 32 48 60; do for b in 4 8 16; do run SVO_REFILL=$r SVO_BLOCKS_PER_CU=$b || exit $?; done; done
