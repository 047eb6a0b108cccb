#!/bin/bash
# Round 4: tools-build bench lines, one per knob set.  usage: bash tools/r4_sweep.sh TAG "K=V K=V" "K=V" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; mkdir -p $O
T=$1; shift
bline() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(sys.argv[2], d["value"], d["ms_per_step"], "enc", p["encoder"]["ms_per_step"], "dec", p["decode"]["ms_per_step"])' $1 "$2"; }
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('tools/libicap_tools.so')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '10', '--warmup', '2']
runpy.run_path('bench.py', run_name='__main__')
" > $O/${T}_b.json 2> $O/${T}_b.err || { tail -20 $O/${T}_b.err; exit 1; }
  bline $O/${T}_b.json "$cfg"
done
