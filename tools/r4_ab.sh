#!/bin/bash
# Round 4 A/B on one box: the product build (new forms on) against the tools build with one form switched back by its
# knob; then a kernel trace of the product bench's decode.  usage: bash tools/r4_ab.sh TAG "KNOB=0 ..." [TESTS]
# OLD_LIB: the old arm's library (default the tools build; a product build of an earlier tree compares like with like -
# the tools build carries the tools-only paths inside the decode kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; mkdir -p $O
T=${1:-ab}
if [ -n "$3" ]; then
  timeout -k 10 400 python -u -m pytest $3 -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
  tail -1 $O/${T}_tests.log
fi
bline() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(sys.argv[2], d["value"], d["ms_per_step"], "enc", p["encoder"]["ms_per_step"], "dec", p["decode"]["ms_per_step"])' $1 $2; }
for v in ${ARMS:-new old new old}; do
  if [ $v = new ]; then
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 $BENCH_ARGS > $O/${T}_b.json 2> $O/${T}_b.err || { tail -20 $O/${T}_b.err; exit 1; }
  else
    OL=${OLD_LIB:-tools/libicap_tools.so}
    env $2 BENCH_LIB=$OL timeout -k 10 200 python -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('$OL')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '10', '--warmup', '2'] + '$BENCH_ARGS'.split()
runpy.run_path('bench.py', run_name='__main__')
" > $O/${T}_b.json 2> $O/${T}_b.err || { tail -20 $O/${T}_b.err; exit 1; }
  fi
  bline $O/${T}_b.json $v
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $O/${T}_prof.log 2>&1 || exit 1
f=$(find $O/${T}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_decode.py $f > $O/${T}_decode_trace.txt 2>&1
cp $(find $O/${T}_prof -name "*kernel_stats.csv" | head -1) $O/${T}_kernel_stats.csv
rm -f $f
head -16 $O/${T}_decode_trace.txt
