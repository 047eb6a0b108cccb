#!/bin/bash
# timing ablations of the persistent fp16 GEMM (tools build): full kernel, no k-loop DMA, no MFMA; the four ViT shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 400 python -m image_caption_amd.build --tools > gpurun_out/r2/ab_build.log 2>&1 || { tail -5 gpurun_out/r2/ab_build.log; exit 1; }
for a in 0 1 2; do
  echo "== ICAP_F16P_ABL=$a (ICAP_F16_PP=0)"
  ICAP_F16_PP=0 ICAP_F16P_ABL=$a timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done
