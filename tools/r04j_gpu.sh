# round-4 final-tree evidence (TAG=r04j: after the per-render marker was dropped; r04k: the moving-camera
# rebuild throttle): GPU suite, smoke,
# the driver's own bench command, then the bench / kernel-trace / PMC passes that
# tools/pmc_summary.py turns into profiles/pmc_summary.json for this tree's digest
export TMPDIR=/tmp
TAG=${TAG:-r04j}
bash tools/gpu_steps.sh gpurun_out/$TAG \
 "600 gputest python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 smoke python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "300 drvplain python3 bench.py --gpus 1 --steps 20 --warmup 5" || exit $?
bash tools/gpu_bench_profile.sh $TAG
