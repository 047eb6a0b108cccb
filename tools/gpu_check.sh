#!/bin/bash
# One GPU round-trip: parity tests, bench line, rocprofv3 kernel trace of the bench + decode breakdown.
# usage: bash tools/gpu_check.sh [tag]
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t_$tag.log 2>&1
st=$?; tail -3 gpurun_out/t_$tag.log; [ $st -eq 0 ] || exit $st
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/b_$tag.log 2>&1 || exit $?
tail -1 gpurun_out/b_$tag.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pb_$tag.log 2>&1 || exit $?
f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
python tools/trace_decode.py $f > gpurun_out/trace_$tag.txt 2>&1
cat gpurun_out/trace_$tag.txt
