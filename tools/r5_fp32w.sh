#!/bin/bash
# Round 5: hi/lo decoder weights (fp32 checkpoints) through the fused blocks - GPU tests, then bench lines with
# --fp32-weights (greedy, beam 5) and the bf16-exact default, on this tree's library against OLD_LIB.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5; mkdir -p $O
T=${1:-w}; OLD=${OLD_LIB:-tools/ab/libicap_base.so}
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -q -s --timeout 200 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
  grep -E "fp32 weights|config2 fp32|passed|failed" $O/${T}_tests.log | tail -5
fi
for args in "--fp32-weights" "--fp32-weights --mode beam" ""; do
  for L in image_caption_amd/libicap.so $OLD; do
    timeout -k 10 200 python -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('$L')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '10', '--warmup', '2'] + '$args'.split()
runpy.run_path('bench.py', run_name='__main__')
" > $O/${T}_b.json 2> $O/${T}_b.err || { tail -20 $O/${T}_b.err; exit 1; }
    python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"].get("phases",{}); print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], "dec", p.get("decode",{}).get("ms_per_step"))' $O/${T}_b.json "$(basename $L)" "$args" | tee -a $O/${T}_ab.txt
  done
done
