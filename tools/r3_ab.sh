#!/bin/bash
# Round 3 (tools build in-tree): same-box A/B of one knob on the ViT and Grid benches, alternating.
# usage: KNOB=ICAP_X VALUES="1 0 1 0" bash tools/r3_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in ${VALUES:-1 0 1 0}; do
  for m in ${MODELS:-vit grid}; do
    r=$(timeout -k 10 150 env $KNOB=$v python bench.py --model $m --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])') || exit 1
    echo "$KNOB=$v $m: $r"
  done
done
