#!/bin/bash
# Round 3 (tools build in-tree): the fp16 trunk convolutions with N % 256 == 0 on the 64-deep k-loop (ICAP_GEMM_C3).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
for v in ${FORMS:-1 2 3 11}; do
  timeout -k 10 300 env ICAP_GEMM_C3=$v python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k grid > $O/c3_tests_$v.log 2>&1 || { tail -30 $O/c3_tests_$v.log; exit 1; }
  echo "form $v: $(tail -1 $O/c3_tests_$v.log)"
done
for v in 0 ${FORMS:-1 2 3 11}; do
  echo "== ICAP_GEMM_C3=$v"
  timeout -k 10 150 env ICAP_GEMM_C3=$v python bench.py --model grid --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"])' || exit 1
  timeout -k 10 200 env ICAP_GEMM_C3=$v rocprofv3 --kernel-trace --output-format csv -d $O/c3_$v -o run -- python3 bench.py --model grid --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find $O/c3_$v -name "*kernel_trace.csv" | head -1)
  python3 tools/trunk_breakdown.py $f > $O/c3_trunk_$v.txt
  grep -E "c3|l3c1|l3c2|total" $O/c3_trunk_$v.txt
  rm -rf $O/c3_$v
done
