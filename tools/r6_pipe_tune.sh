#!/bin/bash
# Round 6: the pipelined bench under an encoder CU budget (persistent encoder grids on fewer CUs, no mask, so decode
# workgroups find free CUs) and with the priorities swapped; alternating runs on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O; : > $O/pipe_tune.txt
# R6_PT_SET="a,b c,d": variants as enc_cus,priority pairs
for r in 1 2; do
  for v in ${R6_PT_SET:-"0 -1" "248 -1" "240 -1" "224 -1" "0 0"}; do
    set -- ${v/,/ }
    ICAP_PIPE_ENC_CUS=$1 ICAP_PIPE_DECODE_PRIORITY=$2 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/pt.json 2> $O/pt.err || { tail -20 $O/pt.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/pt.json')); p=d['roofline']['phases']; print('enc_cus=$1 prio=$2', d['value'], d['ms_per_step'], p['encoder']['ms_per_step'], p['decode']['ms_per_step'])" | tee -a $O/pipe_tune.txt
  done
done
