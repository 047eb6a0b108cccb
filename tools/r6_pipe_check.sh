#!/bin/bash
# Round 6: the pipelined bench default - the ViT line (with the CPU baseline), the Grid line, the sequential line, the
# pipeline test, and the N = 2 flow rehearsed on one GPU (gloo, every rank on cuda:0).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_2_engine.py -x -q --timeout 150 --timeout-method thread -k "pipeline or profile" > $O/pc_tests.log 2>&1 || { tail -20 $O/pc_tests.log; exit 1; }
tail -1 $O/pc_tests.log
timeout -k 10 300 python bench.py > $O/pc_vit.json 2> $O/pc_vit.err || { tail -20 $O/pc_vit.err; exit 1; }
tail -1 $O/pc_vit.json
timeout -k 10 300 python bench.py --model grid --no-cpu-baseline > $O/pc_grid.json 2> $O/pc_grid.err || { tail -20 $O/pc_grid.err; exit 1; }
tail -1 $O/pc_grid.json | cut -c1-300
timeout -k 10 300 python bench.py --sequential --no-cpu-baseline > $O/pc_seq.json 2> $O/pc_seq.err || { tail -20 $O/pc_seq.err; exit 1; }
tail -1 $O/pc_seq.json | cut -c1-300
BENCH_DIST_BACKEND=gloo BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/pc_dist2.json 2> $O/pc_dist2.err || { tail -30 $O/pc_dist2.err; exit 1; }
tail -1 $O/pc_dist2.json | cut -c1-400
