#!/bin/bash
# Encoder attention counters (SQ passes over the ViT encoder, B = 256) for the product library and a variant:
# usage: bash tools/r5_attn_pmc.sh VARIANT.so
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for lib in $R/image_caption_amd/libicap.so $R/$1; do
  n=$(basename $lib .so)
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    ICAP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/r5/apmc_${n}_$i -o run -- python3 $R/tools/encode_grid.py 2 256 vit > $R/gpurun_out/r5/apmc_${n}_$i.log 2>&1 || exit 1
  done
  cd $R && for d in gpurun_out/r5/apmc_${n}_*; do [ -d $d ] && python3 tools/pmc_summary.py $d; done 2>&1 | grep -A 24 "enc_attention" | grep -v "^--" > gpurun_out/r5/apmc_$n.txt
  find gpurun_out/r5 -path "*apmc_*" -name "*.csv" -delete
  cd /tmp
done
