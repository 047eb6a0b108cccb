#!/bin/bash
# Round 6: the f16h GEMM variant against the tree's library on the ViT shapes + edge shapes (tools/r6_gemm_check.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 150 python tools/r6_gemm_check.py > $O/gemm_base.txt 2>&1; rc=$?; cat $O/gemm_base.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit 1
timeout -k 10 150 python tools/r6_gemm_check.py tools/ab/libicap_f16h.so > $O/gemm_f16h.txt 2>&1; rc=$?; cat $O/gemm_f16h.txt | grep -v amdgpu.ids; exit $rc
