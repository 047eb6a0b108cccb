#!/bin/bash
# GEMM tail split: op test, every GPU test, A/B bench (ICAP_GEMM_TAIL=0 vs 1), kernel stats of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_6_ops.py -x -v --timeout 120 --timeout-method thread -k tail_split > gpurun_out/tail_ops.log 2>&1 || { tail -40 gpurun_out/tail_ops.log; exit 1; }
tail -2 gpurun_out/tail_ops.log
timeout -k 10 600 ICAP_GEMM_TAIL=1 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_tests.log 2>&1 || { tail -40 gpurun_out/tail_tests.log; exit 1; }
tail -2 gpurun_out/tail_tests.log
for r in 1 2; do
for k in 0 1; do
timeout -k 10 200 env ICAP_GEMM_TAIL=$k python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/tail_vit_${k}_$r.json 2>gpurun_out/tail.err || exit 1
done
done
for k in 0 1; do
timeout -k 10 200 env ICAP_GEMM_TAIL=$k python bench.py --model grid --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/tail_grid_${k}.json 2>gpurun_out/tail.err || exit 1
done
for f in gpurun_out/tail_vit_*.json gpurun_out/tail_grid_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
export TMPDIR=/tmp
for k in 0 1; do
ICAP_GEMM_TAIL=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tailp_$k -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tailp_$k.log 2>&1 || exit 1
f=$(find gpurun_out/tailp_$k -name "*kernel_stats.csv" | head -1)
echo "== ICAP_GEMM_TAIL=$k"; python3 -c "
import csv
for x in list(csv.DictReader(open('$f')))[:3]: print('%-70s %6s %10.1f us' % (x['Name'][:70], x['Calls'], float(x['AverageNs'])/1e3))
"
done
