#!/bin/bash
# One GPU session: bench (default + overview camera), kernel-trace profile, PMC passes.
# The profiled runs skip the extra camera poses so every primary-ray launch is the bench workload
# (the per-kernel averages then match the bench line's kernel time).
# Usage (inside gpurun): bash tools/gpu_bench_profile.sh <tag>
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 python bench.py --camera overview --cpu-seconds 0 > $OUT/bench_overview.json 2>> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --cpu-seconds 0 --no-extras > $OUT/bench_prof.json 2> $OUT/prof.err || exit $?
# the driver's command (K = 20, W = 5) under the same trace: its kernel_ms against rocprof's mean
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_driver -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-extras > $OUT/bench_driver_prof.json 2> $OUT/prof_driver.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "render_(tile|seg)_kernel" -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > /dev/null 2> $OUT/pmc1.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --kernel-include-regex "render_(tile|seg)_kernel" -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > /dev/null 2> $OUT/pmc2.err || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --kernel-include-regex "render_(tile|seg)_kernel" -d $OUT/pmc_l2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > /dev/null 2> $OUT/pmc3.err || exit $?
echo done
