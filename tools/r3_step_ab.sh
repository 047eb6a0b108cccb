#!/bin/bash
# A/B of the decode loop form: persistent decode step vs one launch per fused block (tools build: ICAP_DEC_STEP),
# headline bench alternating, then a rocprofv3 kernel trace of the persistent form.
# usage: bash tools/r3_step_ab.sh TAG   (outputs under gpurun_out/r3/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-ab}
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 400 python -m image_caption_amd.build --tools > $O/${T}_build.log 2>&1 || { tail -5 $O/${T}_build.log; exit 1; }
for v in 1 0; do
  echo "== ICAP_DEC_STEP=$v"
  ICAP_DEC_STEP=$v timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
for m in "--model grid" "--mode scst --batch 128"; do
  for v in 1 0; do
    echo "== $m ICAP_DEC_STEP=$v"
    ICAP_DEC_STEP=$v timeout -k 10 150 python bench.py --no-cpu-baseline --steps 5 --warmup 2 $m 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"].get("phases", {}).get("decode", {}).get("ms_per_step"))' || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/${T}_prof.log 2>&1 || exit 1
f=$(find $O/${T}_prof -name "*kernel_stats.csv" | head -1)
head -12 $f | cut -d, -f1-8
