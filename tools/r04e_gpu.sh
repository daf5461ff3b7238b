# round-4 final-tree evidence, part 2: the driver's command under a kernel trace, and
# tools/gpu_bench_profile.sh (default bench at K = 1000, overview line, kernel-trace stats of the
# --no-extras run, PMC passes for roofline.traffic)
export TMPDIR=/tmp
TAG=${TAG:-r04e}
bash tools/gpu_steps.sh gpurun_out/$TAG \
 "300 drvtrace rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/drvprof -o drv -- python3 bench.py --gpus 1 --steps 20 --warmup 5" \
 "1000 profile bash tools/gpu_bench_profile.sh $TAG/p"
