# round-4 GPU session h: samples kernel with a non-temporal accumulation store (read keeps the default)
export TMPDIR=/tmp
bash tools/gpu_steps.sh gpurun_out/r04h "300 rehearse python3 tools/samples_rehearsal.py"
