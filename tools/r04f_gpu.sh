# round-4: does a lighter trip (predicated node fetch) hold a higher clock during the ramp?
# launch_series under SVO_FETCH_ALL=1 (default on C3) and =0, interleaved, separate processes
export TMPDIR=/tmp
mkdir -p gpurun_out/r04f
bash tools/gpu_steps.sh gpurun_out/r04f \
 "200 fa1a env SVO_FETCH_ALL=1 python3 tools/launch_series.py --launches 400 --short 100" \
 "200 fa0a env SVO_FETCH_ALL=0 python3 tools/launch_series.py --launches 400 --short 100" \
 "200 fa1b env SVO_FETCH_ALL=1 python3 tools/launch_series.py --launches 400 --short 100" \
 "200 fa0b env SVO_FETCH_ALL=0 python3 tools/launch_series.py --launches 400 --short 100"
bash tools/gpu_steps.sh gpurun_out/r04f "300 rehearse python3 tools/samples_rehearsal.py"
