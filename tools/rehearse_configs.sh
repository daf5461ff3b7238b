#!/bin/bash
# Rehearse the strong-scaling configs C4 (4 GPUs) and C5 (8 GPUs) on a one-GPU box:
#  * ranks: C4 with 4 torchrun ranks sharing cuda:0 over gloo (SVO broadcast from
#    rank 0, band render, host-staged gather, rank 0's assemble, frame check);
#  * multidevice: C5 with one process and an 8-member multi-device context whose
#    members all sit on cuda:0 (8 replicas of the 100.7 M-node pool, xGMI-pull
#    assemble path, frame check);
#  * C5_RANKS=1: C5 also as 8 torchrun ranks over gloo.
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
if [ "${C5_RANKS:-0}" = 1 ]; then
  # C5 as 8 torchrun ranks (pool built on rank 0, broadcast to 7 ranks over gloo): ~3 min
  ( while sleep 20; do date >> $OUT/heartbeat; done ) &
  hb=$!
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29612 bench.py --gpus 8 --config C5 --steps 5 --warmup 2 --payload rgb8 > $OUT/c5_ranks8.json 2> $OUT/c5_ranks8.err
  rc=$?
  kill $hb
  [ $rc = 0 ] || exit $rc
  tail -n 1 $OUT/c5_ranks8.json
fi
echo done
