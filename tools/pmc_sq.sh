#!/bin/bash
# SQ/L2 counters of the primary-ray kernel for the default bench workload; one pass per counter group
# (rocprofv3 does not split counters over passes: <= 8 SQ counters per pass).
#   bash tools/pmc_sq.sh [out_dir] [kernel_regex]     (default gpurun_out/pmc_sq, render_seg_kernel)
set -o pipefail
OUT=${1:-gpurun_out/pmc_sq}; RE=${2:-render_seg_kernel}; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "$RE" -d $OUT/g$i -o run --output-format csv -- python3 bench.py --steps 20 --warmup 400 --cpu-seconds 0 --no-extras > /dev/null 2>> $OUT/err.log || exit $?
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, json, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + '/g*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
res = {k: round(sum(v) / len(v)) for k, v in sorted(agg.items())}
res["launches"] = {k: len(v) for k, v in sorted(agg.items())}
print(json.dumps(res, indent=1))
open(out + '/summary.json', 'w').write(json.dumps(res, indent=1) + "\n")
PY
