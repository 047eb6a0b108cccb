#!/bin/bash
# Round 6: pipelined bench variants alternating on one box.  R6_PV = "label:ENV=.. ENV=..:bench args;label2:..:.."
# (each variant = a label, environment assignments, extra bench.py flags), R6_PV_ROUNDS rounds (default 2);
# R6_PV_LIB: load that library instead of the tree's.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O; : > $O/pipe_var.txt
IFS=';' read -ra VARS <<< "$R6_PV"
for r in $(seq ${R6_PV_ROUNDS:-2}); do
  for v in "${VARS[@]}"; do
    IFS=':' read -r lab envs args <<< "$v"
    if [ -n "$R6_PV_LIB" ]; then  # a library other than the tree's (e.g. the tools build, for ICAP_* knobs)
      env $envs timeout -k 10 200 python -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('$R6_PV_LIB')
sys.argv = ['bench.py', '--no-cpu-baseline'] + '$args'.split()
runpy.run_path('bench.py', run_name='__main__')
" > $O/pv.json 2> $O/pv.err || { tail -20 $O/pv.err; exit 1; }
    else
      env $envs timeout -k 10 200 python bench.py --no-cpu-baseline $args > $O/pv.json 2> $O/pv.err || { tail -20 $O/pv.err; exit 1; }
    fi
    python -c "import json; d=json.load(open('$O/pv.json')); p=d['roofline']['phases']; print('$lab', d['value'], d['ms_per_step'], p['encoder']['ms_per_step'], p['decode']['ms_per_step'])" | tee -a $O/pipe_var.txt
  done
done
