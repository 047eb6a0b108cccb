#!/bin/bash
# Round 5 A/B of product libraries on one box: bench lines alternating over the given .so files, ROUNDS times, then
# (TRACE=1) a kernel trace of the first library's bench decode.  Every arm is a product build (no tools-build paths
# inside the kernels), so a difference is the change under test.
# usage: bash tools/ab_libs.sh TAG ROUNDS LIB1 [LIB2 ...]    BENCH_ARGS: extra bench.py flags   TESTS: pytest files
# run first on LIB1 (the tree's own build, image_caption_amd/libicap.so, unless named)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${ROUND:-r5}; mkdir -p $O
T=$1; R=$2; shift 2
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
  tail -1 $O/${T}_tests.log
fi
bline() { python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"].get("phases") or {}; e=p.get("encoder", {}).get("ms_per_step"); c=p.get("decode", {}).get("ms_per_step"); print(sys.argv[2], d["value"], d["ms_per_step"], "enc", e, "dec", c, "frac", d["roofline"]["frac"])' $1 $2; }
for r in $(seq $R); do
  for L in "$@"; do
    timeout -k 10 200 python -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('$L')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '10', '--warmup', '2'] + '$BENCH_ARGS'.split()
runpy.run_path('bench.py', run_name='__main__')
" > $O/${T}_b.json 2> $O/${T}_b.err || { tail -20 $O/${T}_b.err; exit 1; }
    bline $O/${T}_b.json $(basename $L) | tee -a $O/${T}_ab.txt
  done
done
if [ -n "$TRACE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $O/${T}_prof.log 2>&1 || exit 1
  f=$(find $O/${T}_prof -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_decode.py $f > $O/${T}_decode_trace.txt 2>&1
  cp $(find $O/${T}_prof -name "*kernel_stats.csv" | head -1) $O/${T}_kernel_stats.csv
  rm -f $f
  head -16 $O/${T}_decode_trace.txt
fi
