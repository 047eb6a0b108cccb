#!/bin/bash
# Pipelined bench over decode priority / branch count / CU split (ICAP_PIPE_*), plus the unpipelined line.
# CFGS: configs separated by ';', each "priority branches decode_cus"
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 150 python bench.py --no-cpu-baseline --steps ${STEPS:-10} --warmup 2 "$@" 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"])'; }
echo "== no pipeline"; run || exit 1
IFS=';' read -ra cfgs <<< "${CFGS:--1 1 0;0 1 0;-1 2 0;0 2 0}"
for cfg in "${cfgs[@]}"; do
  set -- $cfg
  echo "== prio=$1 branches=$2 decode_cus=$3"
  ICAP_PIPE_DECODE_PRIORITY=$1 ICAP_DEC_BRANCHES=$2 ICAP_PIPE_DECODE_CUS=$3 run --pipeline || exit 1
done
echo "== no pipeline"; run || exit 1
