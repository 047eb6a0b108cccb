#!/bin/bash
# Round 3 (tools build in-tree): the W-stationary residual conv form (conv_rmw.hip, ICAP_CONV_RMW=1, default) against
# the 64 x 256 tiles (0): Grid GPU tests with it on, then the Grid bench + trunk breakdown, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "grid or conv or trunk" > $O/rmw_tests.log 2>&1 || { tail -30 $O/rmw_tests.log; exit 1; }
echo "tests: $(tail -1 $O/rmw_tests.log)"
for v in ${VARIANTS:-1 0 1 0}; do
  echo "== ICAP_CONV_RMW=$v"
  timeout -k 10 150 env ICAP_CONV_RMW=$v python bench.py --model grid --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"])' || exit 1
  timeout -k 10 200 env ICAP_CONV_RMW=$v rocprofv3 --kernel-trace --output-format csv -d $O/rmw -o run -- python3 bench.py --model grid --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find $O/rmw -name "*kernel_trace.csv" | head -1)
  python3 tools/trunk_breakdown.py $f > $O/rmw_trunk_$v.txt
  grep -E "c3|total" $O/rmw_trunk_$v.txt | cut -c1-5,44-80 | tr '\n' ';'; echo
  rm -rf $O/rmw
done
