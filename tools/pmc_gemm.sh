#!/bin/bash
# PMC passes over tools/gemm_one.py (one counter group per pass; no trace domains with --pmc).
# usage: bash tools/pmc_gemm.sh SHAPE NSPLIT TAG
set -e
export TMPDIR=/tmp
SHAPE=${1:-qkv}; NS=${2:-2}; TAG=${3:-x}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_REQ_sum TCC_EA0_RDREQ_sum TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/gemm_one.py 3 $SHAPE $NS > $OUT/p$i.log 2>&1
done
python3 tools/pmc_summary.py $OUT
