#!/bin/bash
# Round-2 check: full GPU suite, then the headline bench at 1 and 2 decode chains and a kernel trace of the
# 1-chain decode.  usage: bash tools/r2_check.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-x}
mkdir -p gpurun_out/r2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/${T}_tests.log 2>&1 || { tail -30 gpurun_out/r2/${T}_tests.log; exit 1; }
tail -2 gpurun_out/r2/${T}_tests.log
for c in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --decode-chains $c > gpurun_out/r2/${T}_ch$c.json 2> gpurun_out/r2/${T}_ch$c.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof_$T -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --decode-chains 1 > gpurun_out/r2/prof_$T.log 2>&1 || exit 1
f=$(find gpurun_out/r2/prof_$T -name "*kernel_trace.csv" | head -1)
python tools/trace_decode.py $f > gpurun_out/r2/${T}_trace.txt 2>&1
