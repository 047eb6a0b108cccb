#!/bin/bash
# HBM traffic of the bench's kernels: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
# they cannot share a pass on gfx950) over a short bench.py run, summarised per kernel and per launch.
# usage: bash tools/pmc_bench.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-bench}
OUT=gpurun_out/pmcb_$TAG
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1
done
python3 tools/pmc_traffic.py $OUT > $OUT/traffic.json
cat $OUT/traffic.json
