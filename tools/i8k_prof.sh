#!/bin/bash
# Kernel stats of the headline bench with the block-scaled MLP pair on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in 1 0; do
ICAP_I8_MLP2=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/i8kp_$m -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/i8kp_$m.log 2>&1 || exit 1
f=$(find gpurun_out/i8kp_$m -name "*kernel_stats.csv" | head -1)
echo "== ICAP_I8_MLP2=$m"; python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in r[:8]: print('%-60s %6s %10.1f us' % (x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e3))
"
done
