#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
ICAP_DEC_BRANCHES=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_br2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_br2.log 2>&1 || exit $?
python3 $R/tools/trace_overlap.py $R/gpurun_out/prof_br2/run_kernel_trace.csv
