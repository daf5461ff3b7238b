#!/bin/bash
# round-5 GPU session: beam starts -- their parity tests first, then the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_beam.py tests/test_gpu_seg.py > gpurun_out/r05h_beamtest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r05h_beamtest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05h_bench_driver.json 2> gpurun_out/r05h_bench_driver.log || exit 1
SVO_BEAM=0 timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-extras > gpurun_out/r05h_bench_nobeam.json 2>> gpurun_out/r05h_bench_driver.log || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 0 --no-extras > gpurun_out/r05h_bench_beam.json 2>> gpurun_out/r05h_bench_driver.log || exit 1
echo done
