#!/bin/bash
# Effective GPU clock during the encoder GEMM, isolated vs full chip: GRBM_GUI_ACTIVE (cycles) per
# dispatch over the dispatch's duration (kernel trace of the same PMC pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for M in 1024 50432; do
  GEMM_M=$M timeout -k 10 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/clk_$M -o run -- python3 $R/tools/gemm_one.py 6 qkv 2 > $R/gpurun_out/clk_$M.log 2>&1 || { tail -20 $R/gpurun_out/clk_$M.log; exit 1; }
done
ls $R/gpurun_out/clk_1024
