#!/bin/bash
# Round 6: rocprofv3 kernel trace + stats of the default (pipelined) bench; the trace's launches at the bench's timed
# positions against its live events (tools/r6_pipe_prof.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O; rm -rf $O/pp_prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp_prof -o run -- python3 bench.py --no-cpu-baseline > $O/pp_prof.log 2>&1 || { tail -20 $O/pp_prof.log; exit 1; }
f=$(find $O/pp_prof -name "*kernel_trace.csv" | head -1)
python3 tools/r6_pipe_prof.py $f $O/pp_prof.log > $O/pipe_prof_agreement.txt 2>&1
cp $(find $O/pp_prof -name "*kernel_stats.csv" | head -1) $O/pp_kernel_stats.csv
rm -f $f
cat $O/pipe_prof_agreement.txt
