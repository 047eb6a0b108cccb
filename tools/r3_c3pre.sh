#!/bin/bash
# Round 3 (tools build in-tree): same-box A/B of the residual prefetch of the 64-deep conv forms (ICAP_CONV_PRE) and the
# conv tile policy (ICAP_GEMM_C3): variants C3:PRE, Grid bench + trunk breakdown each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 300 env ICAP_CONV_PRE=0 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k grid > $O/c3p_tests.log 2>&1 || { tail -30 $O/c3p_tests.log; exit 1; }
echo "PRE=0: $(tail -1 $O/c3p_tests.log)"
for vp in ${VARIANTS:-0:1 -1:1 -1:0 -1:1 -1:0}; do
  c=${vp%%:*}; p=${vp##*:}
  echo "== ICAP_GEMM_C3=$c ICAP_CONV_PRE=$p"
  timeout -k 10 150 env ICAP_GEMM_C3=$c ICAP_CONV_PRE=$p python bench.py --model grid --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"])' || exit 1
  timeout -k 10 200 env ICAP_GEMM_C3=$c ICAP_CONV_PRE=$p rocprofv3 --kernel-trace --output-format csv -d $O/c3p -o run -- python3 bench.py --model grid --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find $O/c3p -name "*kernel_trace.csv" | head -1)
  python3 tools/trunk_breakdown.py $f > $O/c3p_trunk_${c}_${p}.txt
  grep -E "c3|c1|c2|ds|total" $O/c3p_trunk_${c}_${p}.txt | cut -c1-5,44-75 | tr '\n' ';'; echo
  rm -rf $O/c3p
done
