#!/bin/bash
# Round 6 evidence session (one of two calls): A = the GPU suite, smoke and the bench / profile / PMC
# passes; B = the band-floor decomposition (+ its kernel trace) and the other configs' bench lines.
# Usage (inside gpurun): bash tools/gpu_round6_final.sh A|B <tag>
set -o pipefail
part=$1; TAG=${2:-r06z}; OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$part" = A ]; then
    SVO_BEAM_SWEEP_OUT=$OUT/beam_sweep.json timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 \
        --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || exit 1
    bash tools/gpu_bench_profile.sh $TAG || exit 1
elif [ "$part" = B ]; then
    for n in 1 2 4 8; do
        timeout -k 10 150 python -u tools/band_floor.py --gpus $n --out $OUT/band_floor_$n.json > $OUT/band_floor_$n.txt 2>&1 || exit 1
    done
    rank=$(python -c "import json; print(json.load(open('$OUT/band_floor_8.json'))['slowest_rank'])") || exit 1
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/band_trace -o band -- \
        python3 tools/band_floor.py --gpus 8 --trace-only --rank $rank > $OUT/band_trace.txt 2>&1 || exit 1
    CPU_SECONDS=3 bash tools/configs_bench.sh $TAG || exit 1
fi
echo done
