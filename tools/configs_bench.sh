#!/bin/bash
# One bench line per BASELINE.json config on one GPU (C4/C5 on ONE GPU here;
# their 4/8-GPU split is the driver's multi-GPU run).  Usage: [CPU_SECONDS=5] bash tools/configs_bench.sh <tag>
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
for c in ${CONFIGS:-C1 C2 C4 C5}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-300} --warmup 20 --cpu-seconds ${CPU_SECONDS:-0} > $OUT/config_$c.json 2>> $OUT/configs.err || exit $?
done
echo done
