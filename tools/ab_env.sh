#!/bin/bash
# Bench A/B over env settings: bash tools/ab_env.sh "ENV1=a ENV2=b" "ENV1=c" ... (model via BENCH_ARGS)
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/abe.log 2>&1 || { tail -20 gpurun_out/abe.log; exit 1; }
  echo "[$cfg] $(tail -1 gpurun_out/abe.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"])')"
done
