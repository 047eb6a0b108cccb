#!/bin/bash
# Round 6: the bench's batch-pipelined mode (--pipeline: encode of batch i+1 beside the decode of batch i) against the
# default sequential steps, alternating on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
line() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"], d["ms_per_step"])' $1 $2; }
for r in 1 2 3; do
  for e in "" "--pipeline"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline $e > $O/pipe_b.json 2> $O/pipe_b.err || { tail -20 $O/pipe_b.err; exit 1; }
    line $O/pipe_b.json "x${e}" | tee -a $O/pipe_ab.txt
  done
done
