#!/bin/bash
# fp16 persistent GEMM, A-fragment reads pipelined PF ahead (tools build, ICAP_F16P_ABL 3: PF 2, 4: PF 3) vs as built.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 400 python -m image_caption_amd.build --tools > gpurun_out/r2/ab_build.log 2>&1 || { tail -5 gpurun_out/r2/ab_build.log; exit 1; }
for a in ${ABLS:-0 3 4 0}; do
  echo "== ICAP_F16P_ABL=$a"
  ICAP_F16P_ABL=$a timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids | cut -c1-60 || exit 1
done
