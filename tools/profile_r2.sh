#!/bin/bash
# Round-2 profile checkpoint of the headline bench: PMC traffic passes (-> profiles/r02/pmc_traffic.json, read by
# bench.py), the bench line with the CPU baseline, rocprofv3 --kernel-trace --stats with the decode breakdown,
# and the bench lines of the other configurations (Grid, SCST reward step, beam 5).
# usage: bash tools/profile_r2.sh TAG    (outputs under gpurun_out/r2/; copy what is judged into profiles/r02/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-fin}
O=gpurun_out/r2
mkdir -p $O
bash tools/pmc_bench.sh $T > $O/${T}_pmc.log 2>&1 || { tail -20 $O/${T}_pmc.log; exit 1; }
cp gpurun_out/pmcb_$T/traffic.json profiles/r02/pmc_traffic.json
cp gpurun_out/pmcb_$T/traffic.json $O/${T}_pmc_traffic.json
timeout -k 10 300 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -20 $O/${T}_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$T.log 2>&1 || exit 1
f=$(find $O/prof_$T -name "*kernel_trace.csv" | head -1)
python tools/trace_decode.py $f > $O/${T}_trace.txt 2>&1
cp $(find $O/prof_$T -name "*kernel_stats.csv" | head -1) $O/${T}_kernel_stats.csv
for cfg in "--model grid" "--mode scst --batch 128" "--mode beam"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline $cfg >> $O/${T}_configs.jsonl 2>> $O/${T}_configs.err || { tail -20 $O/${T}_configs.err; exit 1; }
done
tail -1 $O/${T}_bench.json
cat $O/${T}_configs.jsonl
