#!/bin/bash
# Occupancy sweep of the render kernel (diagnostics, one gpurun call): the same
# library with SVO_LDS_PAD extra LDS bytes per one-wave workgroup, so fewer waves
# fit per CU (160 KB LDS / (5,120 B stack + pad)); C3 flyover kernel time per
# setting.  How much the frame gains from each extra resident wave says how far
# the kernel is from its issue limit.
#   bash tools/occupancy_sweep.sh > gpurun_out/occupancy.txt
set -o pipefail
mkdir -p gpurun_out/occ
# waves/CU:   32   28  24   20   16   12   8
for pad in 0 600 1500 2700 4600 7500 13100; do
  SVO_LDS_PAD=$pad timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-extras \
    > gpurun_out/occ/out.json 2>>gpurun_out/occ/err.log || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/occ/out.json')); lds=5120+$pad; print('pad', $pad, 'waves/CU', min(32, 163840 // lds), 'kernel_ms', d['roofline']['kernel_ms'], 'Mrays/s', d['value'])"
done
