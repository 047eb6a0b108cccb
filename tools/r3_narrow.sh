#!/bin/bash
# Round 3 (tools build in-tree): the 256-family k-loop for the fp16 trunk's narrow convolutions (ICAP_GEMM_NARROW
# 1 = 256-row tiles, 2 = 128-row, 3 = 256 x 64 with 3 stages) - Grid GPU tests per form, then the Grid bench + trunk
# breakdown per form (0 = the 64 x 64 kernel).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
for v in ${FORMS:-1 2 3 4}; do
  timeout -k 10 300 env ICAP_GEMM_NARROW=$v python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k grid > $O/nw_tests_$v.log 2>&1 || { tail -30 $O/nw_tests_$v.log; exit 1; }
  echo "form $v: $(tail -1 $O/nw_tests_$v.log)"
done
for v in 0 ${FORMS:-1 2 3 4}; do
  echo "== ICAP_GEMM_NARROW=$v"
  timeout -k 10 150 env ICAP_GEMM_NARROW=$v python bench.py --model grid --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"])' || exit 1
  timeout -k 10 200 env ICAP_GEMM_NARROW=$v rocprofv3 --kernel-trace --output-format csv -d $O/nw_$v -o run -- python3 bench.py --model grid --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find $O/nw_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/trunk_breakdown.py $f > $O/nw_trunk_$v.txt
  grep -E "stem|l1c1|l1c2|l2c1|l2c2|total" $O/nw_trunk_$v.txt
  rm -rf $O/nw_$v
done
