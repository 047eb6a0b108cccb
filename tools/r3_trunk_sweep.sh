#!/bin/bash
# Round 3 (tools build in-tree): Grid trunk GEMM form per K - ICAP_GEMM_TALL_MIN_K (the smallest K of the 128 x 256
# two-block form; below it 256 x 256 / 16 waves) and ICAP_CONV_CLASS - with the per-convolution breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3
for v in "ICAP_GEMM_TALL_MIN_K=128" "ICAP_GEMM_TALL_MIN_K=512" "ICAP_GEMM_TALL_MIN_K=2048"; do
  echo "== $v"
  timeout -k 10 150 env $v python bench.py --model grid --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"])' || exit 1
  n=$(echo $v | tr '=' '_')
  timeout -k 10 200 env $v rocprofv3 --kernel-trace --output-format csv -d $O/ts_$n -o run -- python3 bench.py --model grid --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find $O/ts_$n -name "*kernel_trace.csv" | head -1)
  python3 tools/trunk_breakdown.py $f | grep -E "l1c3|l2c3|l3c3|l3c1|l3c2|l4c3|total"
  rm -rf $O/ts_$n
done
