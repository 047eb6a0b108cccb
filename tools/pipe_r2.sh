#!/bin/bash
# batch pipelining (bench.py --pipeline) against the default on the round-2 product build, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
for m in default pipe default pipe; do
  if [ $m = pipe ]; then A="--pipeline"; else A=""; fi
  echo "== $m"
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 $A 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' || exit 1
done
