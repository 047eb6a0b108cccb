#!/bin/bash
# Round 6: the bench's N > 1 flow on the final tree (pipelined default) rehearsed on one GPU - 2 and 4 ranks on cuda:0,
# gloo collectives (BENCH_DIST_BACKEND / BENCH_ONE_DEVICE), value null by design.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
for n in 2 4; do
  BENCH_DIST_BACKEND=gloo BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 3 --warmup 1 --no-cpu-baseline > $O/dist${n}_final.json 2> $O/dist${n}_final.err || { tail -30 $O/dist${n}_final.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/dist${n}_final.json').read().strip().splitlines()[-1]); print($n, d['n_gpus'], d['value'], d['config']['pipelined'], d['config']['multi_gpu_check'])"
done
