#!/bin/bash
# Round 6: bench lines with the launch timing of every encoder layer (--prof-every 1, the round-5 bench) against
# layers 0 and 6 only (the default), alternating on one box.  (profiles/r06/sync_steps_ab.txt came from a variant of
# this script over a bench flag, --sync-steps, removed with the deferred stop-rule loop it switched off.)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
line() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"].get("phases") or {}; print(sys.argv[2], d["value"], d["ms_per_step"], "enc", p.get("encoder", {}).get("ms_per_step"), "dec", p.get("decode", {}).get("ms_per_step"), "frac", d["roofline"]["frac"], "avg_us", d["roofline"]["avg_launch_us"])' $1 $2; }
for r in 1 2 3; do
  for e in 1 0; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --prof-every $e > $O/pab_b.json 2> $O/pab_b.err || { tail -20 $O/pab_b.err; exit 1; }
    line $O/pab_b.json every$e | tee -a $O/prof_every_ab.txt
  done
done
