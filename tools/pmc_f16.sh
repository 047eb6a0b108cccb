#!/bin/bash
# PMC passes (one counter group per pass, no trace domains) over one fp16 ViT GEMM shape: ours vs hipBLASLt.
# usage: bash tools/pmc_f16.sh SHAPE TAG
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
SHAPE=${1:-qkv}; TAG=${2:-x}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE" \
           "TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCC_REQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 tools/gemm_f16_one.py 3 $SHAPE > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT
