#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/dbs -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/dbs.log 2>&1 || { tail -5 $O/dbs.log; exit 1; }
f=$(find $O/dbs -name "*kernel_trace.csv" | head -1)
python3 tools/r6_dec_by_step.py $f | tee $O/dec_by_step.txt
find $O/dbs -name "*.csv" -delete
