#!/bin/bash
# Round 3 (tools build in-tree): the 256 x 64 tile class for narrow trunk convolutions (ICAP_GEMM_TALL64) - Grid GPU
# tests with it on, then the Grid bench + trunk breakdown with it off and on.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k grid > $O/t64_tests.log 2>&1 || { tail -30 $O/t64_tests.log; exit 1; }
tail -1 $O/t64_tests.log
for v in 0 1; do
  echo "== ICAP_GEMM_TALL64=$v"
  timeout -k 10 150 env ICAP_GEMM_TALL64=$v python bench.py --model grid --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"])' || exit 1
  timeout -k 10 200 env ICAP_GEMM_TALL64=$v rocprofv3 --kernel-trace --output-format csv -d $O/t64_$v -o run -- python3 bench.py --model grid --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find $O/t64_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/trunk_breakdown.py $f > $O/t64_trunk_$v.txt
  grep -E "stem|l1c1|l1c2|l2c1|l2c2|total" $O/t64_trunk_$v.txt
  rm -rf $O/t64_$v
done
