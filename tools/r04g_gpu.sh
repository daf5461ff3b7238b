# round-4 GPU session g: RGB24 readback tests and A/B, the driver sequence's clock (fixed sampler sync)
export TMPDIR=/tmp
bash tools/gpu_steps.sh gpurun_out/r04g \
 "300 tasync python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py tests/test_c_host.py -k 'async or progressive'" \
 "300 readback python3 tools/readback_ab.py" \
 "300 series python3 tools/launch_series.py --launches 1000 --short 200"
