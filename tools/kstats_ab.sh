#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats of a short bench) for several product libraries on one
# box.  usage: bash tools/kstats_ab.sh TAG LIB1 LIB2 ...   BENCH_ARGS: extra bench flags
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5; mkdir -p $O
T=$1; shift
export TMPDIR=/tmp
for L in "$@"; do
  n=$(basename $L .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_$n -o run -- python3 -c "
import sys, runpy
sys.path.insert(0, '.')
from image_caption_amd import _lib
_lib.load('$L')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '3', '--warmup', '1'] + '$BENCH_ARGS'.split()
runpy.run_path('bench.py', run_name='__main__')
" > $O/${T}_$n.log 2>&1 || { tail -5 $O/${T}_$n.log; exit 1; }
  cp $(find $O/${T}_$n -name "*kernel_stats.csv" | head -1) $O/${T}_${n}_stats.csv
  find $O/${T}_$n -name "*kernel_trace.csv" -delete
done
python3 - $O $T "$@" <<'PY'
import csv, os, sys
O, T, libs = sys.argv[1], sys.argv[2], sys.argv[3:]
tabs = []
for L in libs:
    n = os.path.basename(L)[:-3]
    d = {}
    for r in csv.DictReader(open(f"{O}/{T}_{n}_stats.csv")):
        d[r["Name"][:60]] = (int(r["Calls"]), float(r["AverageNs"]) / 1000)
    tabs.append(d)
keys = sorted(tabs[0], key=lambda k: -tabs[0][k][0] * tabs[0][k][1])[:16]
print("kernel".ljust(62), "  ".join(os.path.basename(L)[:-3][:14].rjust(14) for L in libs))
for k in keys:
    print(k.ljust(62), "  ".join(f"{t[k][1]:14.2f}" if k in t else " " * 14 for t in tabs))
PY
