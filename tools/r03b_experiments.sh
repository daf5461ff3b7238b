#!/bin/bash
# Round-3 diagnostics in one gpurun call (each step under its own time limit,
# stop at the first failure): the C3 pool for CPU-side models, the occupancy
# sweep, the dispatch-order A/B, and the heaviest-wave bound of the strong
# splits (C3 flyover, C5 overview and terrain-facing).
set -o pipefail
out=gpurun_out/r03b
mkdir -p $out
timeout -k 10 120 python tools/dump_pool.py --config C3 --out $out/c3_pool.npz || exit $?
timeout -k 10 300 bash tools/occupancy_sweep.sh > $out/occupancy.txt 2>&1 || exit $?

timeout -k 10 200 python tools/wave_log.py --config C3 --tile-row -2 --out $out/wl.bin > $out/wl_c3_heaviest_row.txt 2>&1 || exit $?
timeout -k 10 200 python tools/wave_log.py --config C3 --out $out/wl.bin > $out/wl_c3_frame.txt 2>&1 || exit $?
timeout -k 10 300 python tools/wave_log.py --config C5 --camera overview --tile-row -2 --out $out/wl.bin > $out/wl_c5_overview_heaviest_row.txt 2>&1 || exit $?
timeout -k 10 300 python tools/wave_log.py --config C5 --camera terrain --tile-row -2 --out $out/wl.bin > $out/wl_c5_terrain_heaviest_row.txt 2>&1 || exit $?
rm -f $out/wl.bin
