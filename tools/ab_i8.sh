#!/bin/bash
# End-to-end A/B of the int8 GEMM forms on the headline bench (ViT, B=256, i8x2).
set -o pipefail
cd $GRAFT_REPO_ROOT
for V in "ICAP_I8_TILE=128" "ICAP_I8_TILE=256"; do
  echo "== $V $(env $V timeout -k 10 300 python bench.py --steps 10 --warmup 3 2>gpurun_out/ab_i8.err | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])')" || exit 1
done
