#!/bin/bash
# fp16 GEMM forms on square shapes (tools build) - the k-loop without the ViT shapes' short K.
set -o pipefail
cd $GRAFT_REPO_ROOT
for n in 4096 8192; do
  for f in 0 1 2 5; do
    echo "== SQUARE=$n ICAP_F16_GEMM=$f"
    SQUARE=$n GEMM_M=$n ICAP_F16_GEMM=$f timeout -k 10 120 python tools/gemm_f16.py 10 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
