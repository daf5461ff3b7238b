#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box.
#  * ranks: 2 torchrun ranks share cuda:0 over gloo (SVO_BENCH_BACKEND=gloo; the
#    driver's multi-GPU runs use RCCL, one GPU per rank): band render, the
#    double-buffered gather to rank 0 (host-staged on gloo) and rank 0's
#    svo_assemble_frame, for both payloads;
#  * multidevice: one process, a multi-device context whose members all sit on
#    cuda:0 (--devices 0,0): band render per member, xGMI-pull assemble.
# Plumbing only: the ranks time-slice one GPU, so the rates are not meaningful.
set -o pipefail
mkdir -p gpurun_out/ranks
export SVO_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
port=29531
for n in ${RANKS:-2}; do
for payload in ${PAYLOADS:-auto rgb8 rgba8 compact sparse}; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $n --steps 10 --warmup 2 --payload $payload > gpurun_out/ranks/out_${n}_$payload.json 2>>gpurun_out/ranks/err.log || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/ranks/out_${n}_$payload.json').read().strip().splitlines()[-1]); print('ranks $n $payload', d['n_gpus'], d['value'], d['scaling'], d['config']['parallelism'], d['roofline']['kernel_ms'], d['multi_gpu'])"
done
done
for n in ${MD_DEVICES-2 4}; do
  devs=$(python3 -c "print(','.join(['0'] * $n))")
  timeout -k 10 300 python bench.py --gpus $n --devices $devs --steps 20 --warmup 3 > gpurun_out/ranks/md_$n.json 2>>gpurun_out/ranks/err.log || exit $?
  cat gpurun_out/ranks/md_$n.json
done
