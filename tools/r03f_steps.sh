#!/bin/bash
# Round-3 check of the event-gated loop-form choice: parity tests, the decision trace across
# pose jumps, and the default bench line (extras and CPU baseline included).
set -o pipefail
o=gpurun_out/r03f; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread > $o/gputest.txt 2>&1 || exit $?
timeout -k 10 120 python tools/lat_debug.py > $o/lat_debug.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py > $o/bench_n1.json 2> $o/bench_err.txt || exit $?
