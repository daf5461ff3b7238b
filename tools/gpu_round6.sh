#!/bin/bash
# Round 6 evidence steps, one GPU session; each step under its own time limit, chained so that a
# failure ends the session.  Usage: bash tools/gpu_round6.sh <step> [tag]
set -o pipefail
step=$1; tag=${2:-r06}
out=gpurun_out/$tag
mkdir -p "$out"
dropin() {   # the drop-in loop (held / jittered / pan) under one svo_config
    local name=$1; shift
    timeout -k 10 150 python -u tools/dropin_loop.py --poses flyover,main "$@" > "$out/dropin_$name.txt" 2>&1
}
bench_lib() {   # the default bench line (no extras) with a given library build
    local name=$1 lib=$2
    SVO_RT_LIB=$lib timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 --steps 1000 --warmup 50 \
        > "$out/bench_$name.json" 2> "$out/bench_$name.err"
}
case $step in
policy)
    dropin default && dropin jit1 --set seg_jitter=1 && dropin jit0 --set seg_jitter=0 &&
    dropin ord1 --set order_every=1 && dropin iss44 --set seg_table_issue=0x44 && dropin noseg --set segments=0 ;;
occupancy)
    lib8=$PWD/raytracingtest_amd/libsvo_rt.so; lib7=$PWD/build/ab/seg7/libsvo_rt.so
    bench_lib w8a "$lib8" && bench_lib w7a "$lib7" && bench_lib w8b "$lib8" && bench_lib w7b "$lib7" ;;
r05ab)
    # the round-5 tree (build/ab/r05tree, its own bench.py and libraries) against this one, and the
    # unbounded-occupancy segmented kernel (seg7), interleaved, on the configs the round-5 table lists
    one() { local name=$1 dir=$2 lib=$3; shift 3
            (cd "$dir" && SVO_RT_LIB=$lib timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 "$@") \
                > "$out/ab_$name.json" 2> "$out/ab_$name.err"; }
    r6=$PWD; r5=$PWD/build/ab/r05tree; l6=$r6/raytracingtest_amd/libsvo_rt.so; l5=$r5/raytracingtest_amd/libsvo_rt.so
    l7=$r6/build/ab/seg7/libsvo_rt.so
    for rep in a b; do
        one c5_r6$rep $r6 $l6 --config C5 --steps 300 --warmup 20 && one c5_r5$rep $r5 $l5 --config C5 --steps 300 --warmup 20 &&
        one c5_w7$rep $r6 $l7 --config C5 --steps 300 --warmup 20 &&
        one c4_r6$rep $r6 $l6 --config C4 --steps 300 --warmup 20 && one c4_r5$rep $r5 $l5 --config C4 --steps 300 --warmup 20 &&
        one ov_r6$rep $r6 $l6 --camera overview && one ov_r5$rep $r5 $l5 --camera overview && one ov_w7$rep $r6 $l7 --camera overview &&
        one fly_r6$rep $r6 $l6 && one fly_r5$rep $r5 $l5 || exit $?
    done ;;
bisect)
    # C4 (one GPU, overview) on the round-5 tree, the round-6 commits touching the kernels, and this
    # tree, interleaved: where the round's C4/C5 slowdown came in (build/ab/t_<commit>)
    one() { local name=$1 dir=$2; shift 2
            (cd "$dir" && timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 --config C4 --steps 300 --warmup 20 "$@") \
                > "$out/bis_$name.json" 2> "$out/bis_$name.err"; }
    for rep in a b; do
        one r05$rep build/ab/r05tree && one 8096f73$rep build/ab/t_8096f73 && one c48f03c$rep build/ab/t_c48f03c &&
        one e8037cc$rep build/ab/t_e8037cc && one head$rep . || exit $?
    done ;;
band)
    timeout -k 10 200 python -u tools/band_floor.py --gpus 8 --out "$out/band_floor_8.json" > "$out/band_floor_8.txt" 2>&1 &&
    timeout -k 10 200 python -u tools/band_floor.py --gpus 4 --out "$out/band_floor_4.json" > "$out/band_floor_4.txt" 2>&1 &&
    rank=$(python -c "import json; print(json.load(open('$out/band_floor_8.json'))['slowest_rank'])") &&
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/band_trace" -o band -- \
        python3 tools/band_floor.py --gpus 8 --trace-only --rank "$rank" > "$out/band_trace.txt" 2>&1 ;;
bandab)
    bf() { local name=$1 n=$2; shift 2
           timeout -k 10 150 python -u tools/band_floor.py --gpus $n --out "$out/bf_${name}_$n.json" "$@" \
               > "$out/bf_${name}_$n.txt" 2>&1; }
    bf default 1 && bf default 8 && bf t4 8 --set seg_table_thin=0x8888 && bf t5 8 --set seg_table_thin=0x88888 &&
    bf t5c 8 --set seg_table_thin=0x88888 --set seg_cap=256 && bf t6c 8 --set seg_table_thin=0x888888 --set seg_cap=512 &&
    bf default 4 && bf l4 4 --set seg_table_latency=0x4444 && bf l5 4 --set seg_table_latency=0x44444 --set seg_cap=256 &&
    bf l8 4 --set seg_table_latency=0x8888 --set seg_cap=256 && bf default 2 && bf l4 2 --set seg_table_latency=0x4444 ;;
jitter)
    timeout -k 10 200 python -u tools/jitter_probe.py > "$out/jitter_probe.txt" 2>&1 &&
    timeout -k 10 200 python -u tools/jitter_probe.py --set cost_history=0 > "$out/jitter_probe_h0.txt" 2>&1 ;;
jitter2)
    j() { local name=$1; shift; timeout -k 10 200 python -u tools/jitter_probe.py "$@" > "$out/jp_$name.txt" 2>&1; }
    j default && j iss8 --set seg_table_issue=0x8 && j jit0 --set seg_jitter=0 && j jit1 --set seg_jitter=1 &&
    j iss48 --set seg_table_issue=0x48 ;;
pantrace)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    for dg in 0 1 2; do
        SVO_BEAM_DIAG=$dg timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$out/pan_diag$dg" -o pan -- \
            python3 tools/moving_camera.py --frames 200 > "$out/pan_diag$dg.txt" 2>&1 || exit 1
    done ;;
bandab2)
    bf() { local name=$1 n=$2; shift 2
           timeout -k 10 150 python -u tools/band_floor.py --gpus $n --out "$out/bf_${name}_$n.json" "$@" \
               > "$out/bf_${name}_$n.txt" 2>&1; }
    bf default 8 && bf t4 8 --set seg_table_thin=0x8888 && bf t48 8 --set seg_table_thin=0x4888 &&
    bf t448 8 --set seg_table_thin=0x44888 --set seg_cap=192 && bf default 4 && bf l48 4 --set seg_table_latency=0x4444 ;;
*) echo "unknown step $step"; exit 2 ;;
esac
