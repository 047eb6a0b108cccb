#!/bin/bash
# Round 3: the group-persistent decode step (xdec.hip) - its equivalence test against the launch loop, then the
# headline bench with the decode loop forms 0 (launch per block) and 2 (group step) alternating, and a rocprofv3
# kernel trace of form 2.  usage: bash tools/r3_xdec.sh TAG   (outputs under gpurun_out/r3/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_2_engine.py -x -v --timeout 120 --timeout-method thread -k "group_decode" > $O/${T}_test.log 2>&1 || { tail -40 $O/${T}_test.log; exit 1; }
tail -6 $O/${T}_test.log
for v in 2 0 2 0; do
  echo "== decode-step $v"
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --decode-step $v 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --decode-step 2 > $O/${T}_prof.log 2>&1 || exit 1
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1)
cp $f $O/${T}_kernel_stats.csv
head -12 $f | cut -d, -f1-8
rm -f $(find $O/${T}_prof -name "*kernel_trace.csv")
