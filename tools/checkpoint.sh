#!/bin/bash
# Checkpoint: the whole GPU suite (-s: the B = 256 greedy counts), smoke, the default bench line (with the CPU
# baseline), the Grid bench line, and a rocprofv3 kernel trace + stats of the ViT bench.  usage: [ROUND=r5] bash tools/checkpoint.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-ck}
O=gpurun_out/${ROUND:-r5}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log; grep "greedy vs oracle" $O/${T}_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -2 $O/${T}_smoke.log
timeout -k 10 400 python bench.py > $O/${T}_vit.json 2> $O/${T}_vit.err || { tail -20 $O/${T}_vit.err; exit 1; }
tail -1 $O/${T}_vit.json
timeout -k 10 300 python bench.py --model grid --no-cpu-baseline > $O/${T}_grid.json 2> $O/${T}_grid.err || { tail -20 $O/${T}_grid.err; exit 1; }
tail -1 $O/${T}_grid.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py ${PROF_ARGS:---steps 3 --warmup 1} --no-cpu-baseline > $O/${T}_prof.log 2>&1 || exit 1
f=$(find $O/${T}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_decode.py $f > $O/${T}_decode_trace.txt 2>&1
cp $(find $O/${T}_prof -name "*kernel_stats.csv" | head -1) $O/${T}_kernel_stats.csv
rm -f $f
tail -12 $O/${T}_decode_trace.txt
