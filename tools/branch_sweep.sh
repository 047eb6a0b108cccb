#!/bin/bash
# Decode chains per batch (ICAP_DEC_BRANCHES) x smallest chain (ICAP_DEC_MIN_ROWS), headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-"2 128" "4 64" "1 128" "4 32"}; do
  set -- $cfg
  echo "== branches=$1 min_rows=$2"
  ICAP_DEC_BRANCHES=$1 ICAP_DEC_MIN_ROWS=$2 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' || exit 1
done
