#!/bin/bash
# Decode self-attention change: every GPU test, bench, kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sa_tests.log 2>&1 || { tail -40 gpurun_out/sa_tests.log; exit 1; }
tail -1 gpurun_out/sa_tests.log
for r in 1 2; do timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sa_vit_$r.json 2>gpurun_out/sa.err || exit 1; tail -1 gpurun_out/sa_vit_$r.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sap -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sap.log 2>&1 || exit 1
f=$(find gpurun_out/sap -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for x in csv.DictReader(open('$f')):
    if 'self_attn' in x['Name'] or 'head_kernel' in x['Name']: print('%-60s %6s %10.2f us' % (x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e3))
"
