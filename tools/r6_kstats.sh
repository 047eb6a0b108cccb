#!/bin/bash
# Round 6: rocprofv3 kernel stats of the bench for each given library (product builds), top kernels printed.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
T=$1; shift
for L in "$@"; do
  n=$(basename $L .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_$n -o run -- python3 -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('$L')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '3', '--warmup', '1']
runpy.run_path('bench.py', run_name='__main__')
" > $O/${T}_$n.log 2>&1 || { tail -5 $O/${T}_$n.log; exit 1; }
  f=$(find $O/${T}_$n -name "*kernel_stats.csv" | head -1)
  cp $f $O/${T}_${n}_kstats.csv
  find $O/${T}_$n -name "*kernel_trace.csv" -delete
  echo "== $n"
  python3 - $f <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:9]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.2f} us")
PY
done
