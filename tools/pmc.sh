#!/bin/bash
# HBM traffic per launch of the bench's kernels (rocprofv3 --pmc, one counter group per pass, no tracing
# domains), ViT and Grid.  usage: [ROUND=r5] [MODELS="vit grid"] [PMC_ARGS="--steps 2 --warmup 1"] bash tools/pmc.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for model in ${MODELS:-vit grid}; do
  OUT=gpurun_out/${ROUND:-r5}/pmc_$model
  mkdir -p $OUT
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --model $model ${PMC_ARGS:---steps 2 --warmup 1} --no-cpu-baseline > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit 1; }
  done
  python3 tools/pmc_traffic.py $OUT > $OUT/traffic.json || exit 1
  find $OUT -name "*counter_collection.csv" -delete
  head -c 600 $OUT/traffic.json; echo
done
