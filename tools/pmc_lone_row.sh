#!/bin/bash
# SQ / cache counters of the render kernel for the lone heaviest tile row and for the whole
# C3 frame (tools/lone_row.py), one rocprofv3 pass per counter group.
# Env: ROWS (default "80 -1"), TAG (output directory under gpurun_out/), and any SVO_* switch.
set -o pipefail
OUT=gpurun_out/${TAG:-pmc_lone}; mkdir -p $OUT; export TMPDIR=/tmp
for what in ${ROWS:-80 -1}; do
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
             "TCP_TOTAL_CACHE_ACCESSES_sum TCC_EA0_RDREQ_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex render_tile_kernel -d $OUT/r${what}_g$i -o run --output-format csv -- python3 tools/lone_row.py --row $what --reps 10 >> $OUT/log.txt 2>> $OUT/err.log || exit $?
  done
done
python3 - <<'PY'
import csv, glob, collections
import os
out = os.environ.get("TAG", "pmc_lone")
for what in os.environ.get("ROWS", "80 -1").split():
    agg = collections.defaultdict(list)
    for f in glob.glob(f'gpurun_out/{out}/r{what}_g*/run_counter_collection.csv'):
        for r in csv.DictReader(open(f)):
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    print("== row" if what != "-1" else "== frame", what)
    for k in sorted(agg): print("  ", k, round(sum(agg[k]) / len(agg[k])))
PY
