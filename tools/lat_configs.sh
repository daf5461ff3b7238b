#!/bin/bash
# Loop form forced each way on the C4 / C5 overview frames (bench.py --no-extras, kernel time).
set -o pipefail
mkdir -p gpurun_out/c45
for c in C4 C5; do for lat in 0 1; do
  SVO_LAT=$lat timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 10 --cpu-seconds 0 --no-extras > gpurun_out/c45/${c}_$lat.json 2>>gpurun_out/c45/err.log || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c45/${c}_$lat.json')); print('$c SVO_LAT=$lat', d['roofline']['kernel_ms'], d['value'])"
done; done
