#!/bin/bash
# Environment A/B inside one gpurun call (same library, separate processes,
# interleaved twice): lone heaviest-row launch time, then the bench's primary
# kernel time, step rate and C3 primary + shadow frame.
#   bash tools/ab_env.sh "SVO_FETCH_ALL=1" "SVO_FETCH_ALL=2" ...
set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for cfg in "$@"; do
    row=$(env $cfg timeout -k 10 200 python tools/wave_log.py --tile-row 80 --out gpurun_out/ab/wl.bin 2>/dev/null | grep uninstrumented) || exit $?
    env $cfg timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 > gpurun_out/ab/out.json 2>>gpurun_out/ab/err.log || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/out.json')); print('$cfg', 'kernel_ms', d['roofline']['kernel_ms'], 'Mrays/s', d['value'], 'shadow_frame_ms', d['c3_plus_shadow_ray']['ms_per_frame'], '| row80', sys.argv[1])" "$row"
  done
done
