#!/usr/bin/env bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: 2 ranks share the GPU
# and their collectives go over gloo (BENCH_DIST_BACKEND); the 8-GPU RCCL run
# is the driver's.  Checks the launch, barrier, max-over-ranks timing,
# gather and the graph-replayed timed loop end to end.  (Config 4's step is
# crc32c_multi_plan over RCCL, which needs one GPU per rank: its one-GPU
# coverage is the self-send GPU test.)
set -u
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 BENCH_DIST_BACKEND=gloo
for cfg in c2 c5; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 2 --steps 10 --warmup 3 --config $cfg --no-cpu --no-host \
      > gpurun_out/dist_$cfg.log 2>&1 || { echo "dist $cfg failed rc=$?"; tail -20 gpurun_out/dist_$cfg.log; exit 1; }
  grep '^{' gpurun_out/dist_$cfg.log | tail -1
done
