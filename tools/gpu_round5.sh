#!/bin/bash
# Round-5 GPU session (tag $1, default r05): the whole GPU suite, the driver's bench command, the
# moving-camera pan, and the segment-table A/B under beam starts.
#   /usr/local/graft/bin/gpurun --timeout 1300 -- 'bash tools/gpu_round5.sh r05o'
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r05}
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${T}_gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${T}_gputest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench_driver.json 2> gpurun_out/${T}_bench_driver.log || exit 1
SVO_MOVE_EVERY=1 timeout -k 10 120 python tools/moving_camera.py > gpurun_out/${T}_moving1.txt 2>&1 || exit 1
SVO_MOVE_EVERY=4 timeout -k 10 120 python tools/moving_camera.py > gpurun_out/${T}_moving4.txt 2>&1 || exit 1
timeout -k 10 500 python tools/seg_ab.py --rounds 1 --timed 150 --cameras flyover,main,overview --variants off+nobeam,auto+nobeam,off,auto,l444+i444,l888+i4 > gpurun_out/${T}_seg_ab.json 2> gpurun_out/${T}_seg_ab.log || exit 1
echo done
