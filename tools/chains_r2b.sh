#!/bin/bash
# Decode chains 3 vs 4 on the current tree (tools build: ICAP_DEC_MIN_ROWS), headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m image_caption_amd.build --tools > gpurun_out/chains_build.log 2>&1 || { tail -5 gpurun_out/chains_build.log; exit 1; }
for cfg in "3 80" "4 64" "3 80" "4 64"; do
  set -- $cfg
  echo "== chains=$1 min_rows=$2"
  ICAP_DEC_MIN_ROWS=$2 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --decode-chains $1 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
