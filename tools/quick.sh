#!/bin/bash
# Quick kernel A/B inside one gpurun call: lone-wave cycles/trip on the heaviest
# tile row, then bench twice.  Usage: bash tools/quick.sh [ENV=..]...
set -o pipefail
mkdir -p gpurun_out
env "$@" timeout -k 10 200 python tools/wave_log.py --tile-row 80 --out gpurun_out/wl_row80.bin 2>/dev/null | grep -E "cycles/trip|span|uninstrumented" || exit $?
for i in 1 2; do
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 > gpurun_out/quick.json 2>>gpurun_out/quick.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/quick.json')); print('bench', d['roofline']['kernel_ms'], d['value'])"
done
