#!/bin/bash
# fp16 GEMM at M = 50432, N = 2304 with K = 768 / 1536 / 3072 (same tiles, longer k-loop): slope = time per
# 64-deep k-step in situ, intercept = per-tile overhead; forms 0 (128x256, 2 blocks/CU) and 5 (256x256).
set -o pipefail
cd $GRAFT_REPO_ROOT
for f in ${KFORMS:-0 5}; do
  for k in 768 1536 3072; do
    SHAPE_NK=2304,$k ICAP_F16_GEMM=$f timeout -k 10 120 python tools/gemm_f16.py 10 2>&1 | grep "TF/s" | sed "s/^/form $f: /" || exit 1
  done
done
