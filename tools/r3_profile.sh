#!/bin/bash
# Round-3 profile checkpoint of the default bench, ViT (headline) and Grid: PMC traffic passes (FETCH_SIZE /
# WRITE_SIZE / MFMA busy: separate rocprofv3 --pmc runs), rocprofv3 --kernel-trace --stats, the decode
# breakdown, and the bench lines.  Outputs under gpurun_out/r3/TAG_*; copy what is judged into profiles/r03/.
# usage: bash tools/r3_profile.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
T=${1:-pf}
O=$R/gpurun_out/r3
mkdir -p $O
export TMPDIR=/tmp
for m in vit grid; do
  P=$O/${T}_pmc_$m
  mkdir -p $P
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $P/p$i -o run -- python3 $R/bench.py --model $m --steps 2 --warmup 1 --no-cpu-baseline > $P/p$i.log 2>&1 || { tail -5 $P/p$i.log; exit 1; }
  done
  python3 tools/pmc_traffic.py $P > $O/${T}_pmc_traffic_$m.json || exit 1
  find $P -name "*counter_collection.csv" -delete
  echo "pmc $m done"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_vit -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/${T}_prof_vit.log 2>&1 || exit 1
f=$(find $O/${T}_prof_vit -name "*kernel_trace.csv" | head -1)
python3 tools/trace_decode.py $f > $O/${T}_decode_trace_vit.txt 2>&1
cp $(find $O/${T}_prof_vit -name "*kernel_stats.csv" | head -1) $O/${T}_kernel_stats_vit.csv
rm -f $f
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof_grid -o run -- python3 $R/bench.py --model grid --steps 3 --warmup 1 --no-cpu-baseline > $O/${T}_prof_grid.log 2>&1 || exit 1
f=$(find $O/${T}_prof_grid -name "*kernel_trace.csv" | head -1)
python3 tools/trunk_breakdown.py $f > $O/${T}_trunk_grid.txt 2>&1
cp $(find $O/${T}_prof_grid -name "*kernel_stats.csv" | head -1) $O/${T}_kernel_stats_grid.csv
rm -f $f
echo "rocprof done"
