#!/bin/bash
# Round 3: the whole GPU suite, then a rocprofv3 kernel trace of the Grid bench (config 3) with the per-convolution
# trunk breakdown.  usage: bash tools/r3_grid_prof.sh TAG   (outputs under gpurun_out/r3/)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
T=${1:-g}
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
timeout -k 10 300 python bench.py --model grid --steps 5 --warmup 2 --no-cpu-baseline > $O/${T}_grid.json 2> $O/${T}_grid.err || { tail -30 $O/${T}_grid.err; exit 1; }
tail -1 $O/${T}_grid.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_${T}_grid -o run -- python3 $R/bench.py --model grid --steps 3 --warmup 1 --no-cpu-baseline > $R/$O/${T}_gridprof.log 2>&1 || { tail -30 $R/$O/${T}_gridprof.log; exit 1; }
cd $R
f=$(find $O/prof_${T}_grid -name "*kernel_trace.csv" | head -1)
python tools/trunk_breakdown.py $f > $O/${T}_trunk.txt 2>&1
cp $(find $O/prof_${T}_grid -name "*kernel_stats.csv" | head -1) $O/${T}_grid_kernel_stats.csv
rm -f $f
tail -5 $O/${T}_trunk.txt
