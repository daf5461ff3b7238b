#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/sweep2
run() {
  env "$@" timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-seconds 0 > gpurun_out/sweep2/out.json 2>>gpurun_out/sweep2/err.log || return $?
  python3 -c "import json; d=json.load(open('gpurun_out/sweep2/out.json')); print('$*', d['roofline']['kernel_ms'], d['value'])"
}
run SVO_XCD_REMAP=0 || exit $?
run SVO_XCD_REMAP=1 || exit $?
run SVO_XCD_REMAP=0 || exit $?
run SVO_XCD_REMAP=1 || exit $?
export TMPDIR=/tmp
for remap in 0 1; do
SVO_XCD_REMAP=$remap timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --kernel-trace --kernel-include-regex render_tile -d gpurun_out/sweep2/sq$remap -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > /dev/null 2>> gpurun_out/sweep2/err.log || exit $?
SVO_XCD_REMAP=$remap timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --kernel-include-regex render_tile -d gpurun_out/sweep2/l2$remap -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > /dev/null 2>> gpurun_out/sweep2/err.log || exit $?
done
echo done
