#!/bin/bash
# Round 3 (tools build already in-tree): the group-step equivalence test, the per-phase trace, the bench A/B.
# usage: bash tools/r3_xdec_tools.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-xt}
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_2_engine.py -x -q --timeout 120 --timeout-method thread -k "group_decode" > $O/${T}_test.log 2>&1 || { tail -30 $O/${T}_test.log; exit 1; }
tail -2 $O/${T}_test.log
ICAP_DEC_STEP=2 ICAP_XDEC_TRACE=1 timeout -k 10 200 python tools/xdec_trace.py vit > $O/${T}_trace.txt 2>&1 || { tail -20 $O/${T}_trace.txt; exit 1; }
cat $O/${T}_trace.txt | grep -v amdgpu.ids
for v in 2 0; do
  echo "== decode-step $v"
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --decode-step $v 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
