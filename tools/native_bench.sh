#!/bin/bash
# The metric's frame timed from a plain C host (examples/bench_native.c) beside bench.py's
# default line on the same box: does the C-ABI path without Python reach the same rate?
#   tools/native_bench.sh [out_dir]
set -euo pipefail
OUT=${1:-gpurun_out/native}
mkdir -p "$OUT"
python - "$OUT/cam_flyover.bin" <<'PY'
import sys
sys.path.insert(0, ".")
from tests.test_c_host import _camera_blob
open(sys.argv[1], "wb").write(_camera_blob(1920, 1080))
PY
gcc -O2 -std=c99 -Wall -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include examples/bench_native.c \
    -Lraytracingtest_amd -lsvo_rt -lsvo_build -L/opt/rocm/lib -lamdhip64 -lm \
    -Wl,-rpath,$PWD/raytracingtest_amd -Wl,-rpath,/opt/rocm/lib -o "$OUT/bench_native"
timeout -k 10 120 "$OUT/bench_native" 4 11 "$OUT/cam_flyover.bin" 1920 1080 1000 50 | tee "$OUT/native.json"
timeout -k 10 300 python -u bench.py --no-extras --cpu-seconds 0 | tee "$OUT/bench_py.json"
timeout -k 10 120 "$OUT/bench_native" 4 11 "$OUT/cam_flyover.bin" 1920 1080 1000 50 | tee -a "$OUT/native.json"
