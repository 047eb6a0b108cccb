#!/bin/bash
# Round 3: batch pipelining with the encoder and the decode on disjoint CU sets (ICAP_PIPE_DECODE_CUS = decode CUs;
# the persistent encoder GEMMs sized to the rest, icap_set_encoder_cus), against the default.
# usage: bash tools/r3_pipe.sh [decode CU counts...]
set -o pipefail
cd $GRAFT_REPO_ROOT
bench() {  # $1: env assignments, $2: extra args
  timeout -k 10 200 env $1 python bench.py --no-cpu-baseline --steps 12 --warmup 3 $2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"])'
}
echo "== default"; bench "X=1" "" || exit 1
echo "== pipeline, priority only"; bench "X=1" "--pipeline" || exit 1
for c in ${@:-64 96 128}; do
  echo "== pipeline, decode CUs $c"; bench "ICAP_PIPE_DECODE_CUS=$c" "--pipeline" || exit 1
done
