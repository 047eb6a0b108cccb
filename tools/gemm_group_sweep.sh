#!/bin/bash
# bf16x2 encoder GEMM raster sweep (ICAP_GEMM_GROUP) over the four ViT shapes, then the bench per setting.
set -o pipefail
cd $GRAFT_REPO_ROOT
for G in 0 4 8 16 32; do
  echo "== G=$G"; ICAP_GEMM_GROUP=$G timeout -k 10 120 python tools/gemm_shapes.py 20 2>/dev/null | cut -c1-75 || exit 1
done
for G in ${BENCH_GROUPS:-0 16}; do
  for P in bf16x2 i8x2; do
    echo "== bench G=$G $P"; ICAP_GEMM_GROUP=$G timeout -k 10 200 python bench.py --precision $P --no-cpu-baseline 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])' || exit 1
  done
done
