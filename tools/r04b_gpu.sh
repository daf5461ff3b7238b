# round-4 GPU session b: the new entry points' parity tests, C3 full-frame parity (incl. the
# Main.unity pose), the samples-in-flight rehearsal, a bench with extras, the rank rehearsal
export TMPDIR=/tmp
bash tools/gpu_steps.sh gpurun_out/r04b \
 "200 dump python3 tools/dump_pool.py --out gpurun_out/c3_pool.npz" \
 "300 tnew python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py tests/test_c_host.py -k 'samples or async or progressive'" \
 "400 tfull python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k full_frame_parity" \
 "300 rehearse python3 tools/samples_rehearsal.py" \
 "300 bench python3 bench.py --steps 200 --warmup 20 --cpu-seconds 2" \
 "400 ranks env RANKS='2 4' PAYLOADS=rgb8 MD_DEVICES= bash tools/rehearse_ranks.sh"
