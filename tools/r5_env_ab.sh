#!/bin/bash
# Bench A/B over HIP runtime environment settings (round 5: kernarg placement / graph packet capture for the decode
# graph's launch cost).  usage: bash tools/r5_env_ab.sh ROUNDS "ENV1=a" "ENV2=b" ...   ("-" = the default environment)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5; mkdir -p $O
R=$1; shift
for r in $(seq $R); do
  for cfg in "$@"; do
    e=$cfg; [ "$cfg" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/envab.json 2> $O/envab.err || { tail -20 $O/envab.err; exit 1; }
    echo "[$cfg] $(tail -1 $O/envab.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], "enc", p["encoder"]["ms_per_step"], "dec", p["decode"]["ms_per_step"])')" | tee -a $O/envab.txt
  done
done
