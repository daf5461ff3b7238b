#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: 2 ranks share cuda:0 over gloo
# (SVO_BENCH_BACKEND=gloo; the driver's multi-GPU runs use RCCL, one GPU per rank).
# Plumbing only: two processes time-slice one GPU, so the rates are not meaningful.
# Default split (samples: weak scaling, no collective in the step), bands
# (+ all-gather of the hit records) and samples + accumulate (all-reduce).
set -o pipefail
mkdir -p gpurun_out/ranks
export SVO_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
port=29531
for extra in "" "--split bands" "--accumulate"; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps 10 --warmup 2 $extra > gpurun_out/ranks/out.json 2>>gpurun_out/ranks/err.log || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/ranks/out.json').read().strip().splitlines()[-1]); print('$extra', d['n_gpus'], d['value'], d['scaling'], d['config']['parallelism'], d['roofline']['kernel_ms'], d['roofline']['kernel_ms_max_rank'])"
done
