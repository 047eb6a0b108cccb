#!/bin/bash
# Rehearsal of bench.py's N > 1 flow (torchrun ranks, contiguous shards, barrier + max-over-ranks timing, the
# gathered-ids stop-rule self-check, rank-0 JSON line) on a one-GPU box: 2 ranks on cuda:0 with gloo collectives.
# The throughput of this line means nothing (two ranks share one GPU); the driver measures N = 1..8 on a node.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
BENCH_DIST_BACKEND=gloo BENCH_ONE_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${N:-2} \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus ${N:-2} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${EXTRA} \
  > gpurun_out/r3/dist${N:-2}${TAG}.json 2> gpurun_out/r3/dist${N:-2}${TAG}.err || { tail -30 gpurun_out/r3/dist${N:-2}${TAG}.err; exit 1; }
tail -1 gpurun_out/r3/dist${N:-2}${TAG}.json
