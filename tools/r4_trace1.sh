#!/bin/bash
# Round 4: kernel trace of the tools-build bench decode with the given knobs (default one decode chain).
# usage: bash tools/r4_trace1.sh TAG ["KNOB=V ..."]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; mkdir -p $O
T=${1:-tr}
export TMPDIR=/tmp
cat > /tmp/run_tools_bench.py <<'PY'
import sys, runpy
from image_caption_amd import _lib
_lib.load('tools/libicap_tools.so')
sys.argv = ['bench.py', '--no-cpu-baseline'] + sys.argv[1:]
runpy.run_path('bench.py', run_name='__main__')
PY
export PYTHONPATH=$GRAFT_REPO_ROOT
for kv in ${2:-ICAP_DEC_BRANCHES=1}; do export $kv; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 /tmp/run_tools_bench.py --steps 3 --warmup 1 > $O/${T}_prof.log 2>&1 || { tail -5 $O/${T}_prof.log; exit 1; }
f=$(find $O/${T}_prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_decode.py $f > $O/${T}_decode_trace.txt 2>&1
cp $(find $O/${T}_prof -name "*kernel_stats.csv" | head -1) $O/${T}_kernel_stats.csv
rm -f $f
cat $O/${T}_decode_trace.txt | tail -20
