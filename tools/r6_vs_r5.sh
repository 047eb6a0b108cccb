#!/bin/bash
# Round 6: the final tree against the round-5 final tree (commit 4339005, built in r5tree/ - not part of the
# repository) on one box: default bench lines alternating, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
line() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"].get("phases") or {}; print(sys.argv[2], d["value"], d["ms_per_step"], "enc", p.get("encoder", {}).get("ms_per_step"), "dec", p.get("decode", {}).get("ms_per_step"), "frac", d["roofline"]["frac"])' $1 $2; }
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/r6r5_b.json 2> $O/r6r5_b.err || { tail -20 $O/r6r5_b.err; exit 1; }
  line $O/r6r5_b.json round6 | tee -a $O/r6_vs_r5.txt
  (cd r5tree && timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > ../$O/r6r5_b.json 2> ../$O/r6r5_b.err) || { tail -20 $O/r6r5_b.err; exit 1; }
  line $O/r6r5_b.json round5 | tee -a $O/r6_vs_r5.txt
done
