#!/bin/bash
# Round 4: decode chain count with the register-fragment decode blocks (tools build knobs), then the encoder attention
# timing ablations.  usage: bash tools/r4_chains.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; mkdir -p $O
T=${1:-ch}
bline() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(sys.argv[2], d["value"], d["ms_per_step"], "enc", p["encoder"]["ms_per_step"], "dec", p["decode"]["ms_per_step"])' $1 "$2"; }
for cfg in "ICAP_DEC_BRANCHES=3" "ICAP_DEC_BRANCHES=1" "ICAP_DEC_BRANCHES=2" "ICAP_DEC_BRANCHES=4 ICAP_DEC_MIN_ROWS=16" "ICAP_DEC_BRANCHES=3"; do
  env $cfg timeout -k 10 200 python -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('tools/libicap_tools.so')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '10', '--warmup', '2']
runpy.run_path('bench.py', run_name='__main__')
" > $O/${T}_b.json 2> $O/${T}_b.err || { tail -20 $O/${T}_b.err; exit 1; }
  bline $O/${T}_b.json "$cfg"
done
bash tools/r4_eaf.sh
