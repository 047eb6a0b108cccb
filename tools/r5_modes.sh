#!/bin/bash
# Round 5: the bench lines of the other modes on this tree (ViT / Grid beam 5, SCST reward step at the config-5
# shape, fp32-checkpoint decoder weights greedy / beam 5).  usage: bash tools/r5_modes.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5; mkdir -p $O
T=${1:-modes}
i=0
while read -r name args; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $args > $O/${T}_$name.json 2> $O/${T}_$name.err || { tail -20 $O/${T}_$name.err; exit 1; }
  echo "$name $(tail -1 $O/${T}_$name.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms")')"
done <<LIST
vit_beam5 --mode beam --beam 5 --steps 3 --warmup 1
grid_beam5 --model grid --mode beam --beam 5 --steps 3 --warmup 1
scst_b128 --mode scst --batch 128 --steps 5 --warmup 2
vit_fp32w --fp32-weights --steps 10 --warmup 2
vit_fp32w_beam5 --fp32-weights --mode beam --beam 5 --steps 3 --warmup 1
LIST
