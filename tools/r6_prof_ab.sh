#!/bin/bash
# Round 6: bench lines A/B (first: the stop rule read before the next step is enqueued, --sync-steps; then the
# default deferred read), alternating on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
line() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"].get("phases") or {}; print(sys.argv[2], d["value"], d["ms_per_step"], "enc", p.get("encoder", {}).get("ms_per_step"), "dec", p.get("decode", {}).get("ms_per_step"), "frac", d["roofline"]["frac"], "avg_us", d["roofline"]["avg_launch_us"])' $1 $2; }
for r in 1 2 3; do
  for e in "--sync-steps" ""; do
    timeout -k 10 200 python bench.py --no-cpu-baseline $e > $O/pab_b.json 2> $O/pab_b.err || { tail -20 $O/pab_b.err; exit 1; }
    line $O/pab_b.json "x${e}" | tee -a $O/sync_steps_ab.txt
  done
done
