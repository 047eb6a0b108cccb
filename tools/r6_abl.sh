#!/bin/bash
# Round 6: timing of GEMM library variants on the ViT shapes (tools/r6_gemm_check.py; ablation variants report FAIL
# parity by construction).  usage: bash tools/r6_abl.sh TAG LIB...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
T=$1; shift
for L in "$@"; do
  echo "== $L"
  timeout -k 10 150 python tools/r6_gemm_check.py $L > $O/${T}_$(basename $L).txt 2>&1
  rc=$?
  grep -E "TF/s|per ViT" $O/${T}_$(basename $L).txt
  [ $rc -le 1 ] || { tail -5 $O/${T}_$(basename $L).txt; exit 1; }
done
