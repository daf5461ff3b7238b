# round-4 final-tree evidence, part 1: the whole GPU suite and smoke, then the driver's own
# bench command (plain), under a kernel trace, and the profile / PMC passes
export TMPDIR=/tmp
TAG=${TAG:-r04d}
bash tools/gpu_steps.sh gpurun_out/$TAG \
 "900 gputest python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200 smoke python3 -c 'import __graft_entry__ as g; g.smoke()'" \
 "300 drvplain python3 bench.py --gpus 1 --steps 20 --warmup 5"
