#!/bin/bash
# SQ/L2 counters of the render kernel for the default bench workload; one pass per counter group.
set -o pipefail
OUT=gpurun_out/pmc_sq; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  env "$@" timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex render_tile_kernel -d $OUT/g$i -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-extras > /dev/null 2>> $OUT/err.log || exit $?
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmc_sq/g*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name']; targs = n[n.index('<')+1:n.index('>')].split(',')
        if targs[1].strip() == 'true': continue
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k in sorted(agg): print(k, round(sum(agg[k]) / len(agg[k])))
PY
