#!/bin/bash
# Rehearse the strong-scaling configs C4 (4 GPUs) and C5 (8 GPUs) on a one-GPU box:
#  * ranks: C4 with 4 torchrun ranks sharing cuda:0 over gloo (SVO broadcast from
#    rank 0, band render, host-staged gather, rank 0's assemble, frame check);
#  * multidevice: C5 with one process and an 8-member multi-device context whose
#    members all sit on cuda:0 (8 replicas of the 100.7 M-node pool, xGMI-pull
#    assemble path, frame check).
# Plumbing and parity only: the members time-slice one GPU, so rates are not
# 4- / 8-GPU rates.  Usage (inside gpurun): bash tools/rehearse_configs.sh
set -o pipefail
OUT=gpurun_out/configs_multi
mkdir -p $OUT
export SVO_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 4 --config C4 --steps 10 --warmup 2 > $OUT/c4_ranks4.json 2> $OUT/c4_ranks4.err || exit $?
tail -n 1 $OUT/c4_ranks4.json
timeout -k 10 500 python bench.py --gpus 8 --devices 0,0,0,0,0,0,0,0 --config C5 --steps 10 --warmup 2 \
  > $OUT/c5_md8.json 2> $OUT/c5_md8.err || exit $?
tail -n 1 $OUT/c5_md8.json
echo done
