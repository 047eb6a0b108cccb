#!/bin/bash
# Where the ViT encoder attention kernel's time goes: SQ counter passes over the ViT encoder (B=256).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/apmc_$i -o run -- python3 $R/tools/encode_grid.py 2 256 vit > $R/gpurun_out/apmc_$i.log 2>&1 || exit 1
done
cd $R && for d in gpurun_out/apmc_1 gpurun_out/apmc_2 gpurun_out/apmc_3; do python3 tools/pmc_summary.py $d; done 2>&1 | grep -A 24 "enc_attention_pipe" | head -60
