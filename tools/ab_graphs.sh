#!/bin/bash
# Decode launch path A/B on the headline bench: captured hipGraph vs eager stream launches, 1 / 2 chains.
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 "$@" 2>>gpurun_out/ab_graphs.err | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
for BR in 2 1; do
  echo "== branches=$BR graph   $(ICAP_DEC_BRANCHES=$BR run)" || exit 1
  echo "== branches=$BR eager   $(ICAP_DEC_BRANCHES=$BR run --no-graphs)" || exit 1
done
