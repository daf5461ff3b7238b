# round-4 GPU session c: readback modes, samples kernel with NT accumulation, loop-form
# decisions under a moving camera, the async tests under each readback mode
export TMPDIR=/tmp
bash tools/gpu_steps.sh gpurun_out/r04c \
 "300 readback python3 tools/readback_ab.py" \
 "300 rehearse python3 tools/samples_rehearsal.py" \
 "300 latdebug python3 tools/lat_debug.py" \
 "300 tasync1 env SVO_PIN_PUSH=1 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py tests/test_c_host.py -k 'async or samples'" \
 "300 tasync2 env SVO_PIN_PUSH=2 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py tests/test_c_host.py -k async"
