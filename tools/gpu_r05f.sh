# round-5 GPU session: GPU suite, the driver's bench command, moving camera, segment A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05g_gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r05g_gputest.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05g_bench_driver.json 2> gpurun_out/r05g_bench_driver.log || exit 1
SVO_MOVE_EVERY=1 timeout -k 10 120 python tools/moving_camera.py > gpurun_out/r05g_moving1.txt 2>&1 || exit 1
SVO_MOVE_EVERY=4 timeout -k 10 120 python tools/moving_camera.py > gpurun_out/r05g_moving4.txt 2>&1 || exit 1
timeout -k 10 400 python tools/seg_ab.py --rounds 1 --variants off,auto,l888,l4888,l488,i0,i8 --cameras flyover,main,overview > gpurun_out/r05g_seg_ab.json 2> gpurun_out/r05g_seg_ab.log
