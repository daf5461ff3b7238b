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
logab)
    # C4 and C3 flyover: this tree against itself without the segmented kernel's wave-log stamps
    # (SVO_SEG_LOG=0, build/ab/nolog, nolog7 = also unbounded VGPRs) and the last tree before them
    one() { local name=$1 dir=$2 lib=$3; shift 3
            (cd "$dir" && SVO_RT_LIB=$lib timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 "$@") \
                > "$out/lg_$name.json" 2> "$out/lg_$name.err"; }
    r6=$PWD; l6=$r6/raytracingtest_amd/libsvo_rt.so; ln=$r6/build/ab/nolog/libsvo_rt.so; ln7=$r6/build/ab/nolog7/libsvo_rt.so
    t8=$r6/build/ab/t_8096f73; l8=$t8/raytracingtest_amd/libsvo_rt.so
    for rep in a b; do
        for v in "head $r6 $l6" "nolog $r6 $ln" "nolog7 $r6 $ln7" "t8096 $t8 $l8"; do
            set -- $v
            one c4_$1$rep $2 $3 --config C4 --steps 300 --warmup 20 && one fly_$1$rep $2 $3 || exit $?
        done
    done
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$out/c4prof" -o c4 -- \
        python3 bench.py --no-extras --cpu-seconds 0 --config C4 --steps 100 --warmup 20 > "$out/c4prof.txt" 2>&1 ;;
fixab)
    # the template-flag wave log (this tree) against the last tree before the stamps and round 5's,
    # on the configs that showed the stamps' cost
    one() { local name=$1 dir=$2; shift 2
            (cd "$dir" && timeout -k 10 200 python -u bench.py --no-extras --cpu-seconds 0 "$@") \
                > "$out/fx_$name.json" 2> "$out/fx_$name.err"; }
    for rep in a b; do
        for v in "head ." "t8096 build/ab/t_8096f73" "r05 build/ab/r05tree"; do
            set -- $v
            one c4_$1$rep $2 --config C4 --steps 300 --warmup 20 && one fly_$1$rep $2 && one ov_$1$rep $2 --camera overview &&
            one main_$1$rep $2 --camera main || exit $?
        done
        one c5_head$rep . --config C5 --steps 300 --warmup 20 && one c5_r05$rep build/ab/r05tree --config C5 --steps 300 --warmup 20 || exit $?
    done ;;
sgprab)
    # the segmented kernel's node-pool pointer: reloaded from the kernel arguments every trip (head),
    # pinned in SGPRs (pin), a larger SGPR budget (sgpr80), both (pin80); interleaved
    one() { local name=$1 lib=$2; shift 2
            SVO_RT_LIB=$lib timeout -k 10 200 python -u bench.py --no-extras --cpu-seconds 0 "$@" \
                > "$out/sg_$name.json" 2> "$out/sg_$name.err"; }
    for rep in a b; do
        for v in head:raytracingtest_amd pin:build/ab/pin sgpr80:build/ab/sgpr80 pin80:build/ab/pin80; do
            n=${v%%:*}; l=$PWD/${v#*:}/libsvo_rt.so
            one fly_$n$rep $l && one main_$n$rep $l --camera main && one c4_$n$rep $l --config C4 --steps 300 --warmup 20 || exit $?
        done
    done ;;
sq)
    # SQ issue / wait counters of the segmented kernel (C3 flyover), the segmented parity tests, one
    # wave-logged band (the LOG instantiation)
    timeout -k 10 400 bash tools/pmc_sq.sh "$out/pmc_sq" render_seg_kernel > "$out/pmc_sq.txt" 2>&1 &&
    timeout -k 10 300 python -u -m pytest tests/test_gpu_seg.py -x -q --timeout 120 --timeout-method thread > "$out/seg_tests.txt" 2>&1 &&
    timeout -k 10 200 python -u tools/band_floor.py --gpus 8 --out "$out/band_floor_8.json" > "$out/band_floor_8.txt" 2>&1 ;;
splatab)
    # beam splat workgroup size (SVO_SPLAT_THREADS 512 / 256 / 128): the pan loop's frame and the
    # splat kernel's own time (rocprofv3 kernel trace of the same loop)
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    for rep in a b; do
        for v in ${SPLATS:-512:raytracingtest_amd 256:build/ab/splat256 128:build/ab/splat128}; do
            n=${v%%:*}; l=$PWD/${v#*:}/libsvo_rt.so
            SVO_RT_LIB=$l timeout -k 10 150 python -u tools/dropin_loop.py --poses flyover,main > "$out/sp_$n$rep.txt" 2>&1 || exit $?
        done
    done
    [ -n "$SPLATS" ] && exit 0
    for v in 512:raytracingtest_amd 256:build/ab/splat256 128:build/ab/splat128; do
        n=${v%%:*}; l=$PWD/${v#*:}/libsvo_rt.so
        SVO_RT_LIB=$l timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$out/sp_prof_$n" -o sp -- \
            python3 tools/dropin_loop.py --poses flyover --frames 200 > "$out/sp_prof_$n.txt" 2>&1 || exit $?
    done ;;
backab)
    # splat depth (svo_config.beam_back 2 = default, 3, 4; BACKS overrides): held / jittered / pan frames
    for rep in a b; do
        for v in ${BACKS:-2 3 4}; do
            timeout -k 10 150 python -u tools/dropin_loop.py --poses flyover,main --set beam_back=$v > "$out/bb_$v$rep.txt" 2>&1 || exit $?
        done
    done ;;
progtrace)
    # the shim's per-frame call alone (held fixed / jittered / pan), then under a kernel + copy trace
    timeout -k 10 150 python -u tools/progressive_trace.py > "$out/pt_plain.txt" 2>&1 &&
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
    timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d "$out/pt" -o pt -- \
        python3 tools/progressive_trace.py > "$out/pt_prof.txt" 2>&1 ;;
heldab)
    # a held view's finer re-splat (beam_back_held 0, the default) against none (-1): parity of the
    # beam / segment / decision suites first, then the drop-in loops and the bench line, interleaved
    timeout -k 10 600 python -u -m pytest tests/test_gpu_beam.py tests/test_gpu_seg.py -x -v --timeout 200 \
        --timeout-method thread > "$out/held_tests.txt" 2>&1 &&
    timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
        -k "class_table or loop_form or switches" > "$out/held_tests2.txt" 2>&1 || exit $?
    for rep in a b; do
        for v in 0 -1; do
            timeout -k 10 150 python -u tools/dropin_loop.py --poses flyover,main --set beam_back_held=$v \
                > "$out/hd_$v$rep.txt" 2>&1 || exit $?
            timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 --set beam_back_held=$v \
                > "$out/hb_fly_$v$rep.json" 2> "$out/hb_$v$rep.err" || exit $?
            timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 --camera main --set beam_back_held=$v \
                > "$out/hb_main_$v$rep.json" 2>> "$out/hb_$v$rep.err" || exit $?
        done
    done ;;
tableab)
    # the class tables under the held view's fine starts (bench line, flyover and Main.unity pose)
    one() { local name=$1; shift
            timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 "$@" > "$out/tb_$name.json" 2>> "$out/tb.err"; }
    for rep in a b; do
        for v in ${TABLES:-"default:" "noseg:--set segments=0" "iss44:--set seg_table_issue=0x44" "iss8:--set seg_table_issue=0x8" "cap192:--set seg_cap=192"}; do
            n=${v%%:*}; a=${v#*:}; a=${a//+/ }   # '+' stands for a space inside one TABLES entry
            for pose in ${POSES:-flyover main}; do
                one ${pose:0:4}_$n$rep --camera $pose $a || exit $?
            done
        done
    done ;;
splatcost)
    # the splat kernel's own time per list depth (beam_back 2 / 1 / 0 for the moving camera) over the
    # pan loop, from a kernel trace
    cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
    for v in 2 1 0; do
        timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$out/sc_$v" -o sc -- \
            python3 tools/progressive_trace.py --frames 100 --set beam_back=$v > "$out/sc_$v.txt" 2>&1 || exit $?
    done ;;
jitab)
    # the jittered launch's segment starts under the held view's fine splat (seg_jitter 2 default / 1 / 0)
    for rep in a b; do
        for v in 2 1 0; do
            timeout -k 10 150 python -u tools/dropin_loop.py --poses flyover,main --set seg_jitter=$v > "$out/jt_$v$rep.txt" 2>&1 || exit $?
        done
    done ;;
longab)
    # the long splat list's boxes per thread (SVO_SPLAT_LONG_PER 4 = this tree, 1, 8) on the pan with the
    # moving list at one and zero levels back, and the beam suite on this tree first
    timeout -k 10 400 python -u -m pytest tests/test_gpu_beam.py -x -q --timeout 200 --timeout-method thread \
        > "$out/beam_tests.txt" 2>&1 || exit $?
    for rep in a b; do
        for v in 4:raytracingtest_amd 1:build/ab/long1 8:build/ab/long8; do
            n=${v%%:*}; l=$PWD/${v#*:}/libsvo_rt.so
            for bb in 1 0; do
                SVO_RT_LIB=$l timeout -k 10 150 python -u tools/dropin_loop.py --poses flyover,main --set beam_back=$bb \
                    > "$out/lp_${n}_bb$bb$rep.txt" 2>&1 || exit $?
            done
        done
    done ;;
orderab)
    # the periodic order rebuild while costs drift (order_every 32 default / 16 / 8 / 4) on the drop-in loops
    for rep in a b; do
        for v in ${EVERY:-32 16 8 4}; do
            timeout -k 10 150 python -u tools/dropin_loop.py --poses flyover,main --set order_every=$v > "$out/oe_$v$rep.txt" 2>&1 || exit $?
        done
    done ;;
armab)
    # one compare fewer per trip in the beam loop (arm = not skip): parity first, then interleaved
    timeout -k 10 500 python -u -m pytest tests/test_gpu_beam.py tests/test_gpu_seg.py tests/test_gpu_fullsize.py -x -q \
        --timeout 300 --timeout-method thread > "$out/arm_tests.txt" 2>&1 || exit $?
    for rep in a b c; do
        for v in new:raytracingtest_amd base:build/ab/base; do
            n=${v%%:*}; l=$PWD/${v#*:}/libsvo_rt.so
            SVO_RT_LIB=$l timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 > "$out/am_fly_$n$rep.json" 2>> "$out/am.err" &&
            SVO_RT_LIB=$l timeout -k 10 150 python -u bench.py --no-extras --cpu-seconds 0 --camera main > "$out/am_main_$n$rep.json" 2>> "$out/am.err" || exit $?
        done
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
