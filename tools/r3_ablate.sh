#!/bin/bash
# Round 3 timing ablations of the persistent fp16 GEMM (tools build in-tree): full, no k-loop DMA (1), no MFMA (2), no
# LDS fragment reads (9), no DMA and no k-step barrier (10); the four ViT shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
for a in ${ABLS:-0 1 2 9 10}; do
  echo "== ICAP_F16P_ABL=$a"
  ICAP_F16P_ABL=$a timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done
