#!/bin/bash
# Full GPU suite + headline bench (default precision) + rocprofv3 kernel stats of the bench.
# usage: bash tools/full_check.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/${T}_bench.json 2> $O/${T}_bench.err || exit 1
cat $O/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$T.log 2>&1 || exit 1
f=$(find $O/prof_$T -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 $f | head -22
