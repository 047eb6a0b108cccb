#!/bin/bash
# Profile checkpoint of the headline bench: PMC traffic passes (FETCH_SIZE / WRITE_SIZE / MFMA busy),
# the bench line (reads the fresh traffic table), rocprofv3 --kernel-trace --stats and the decode breakdown.
# usage: bash tools/profile_round.sh TAG   (outputs under gpurun_out/; copy what is judged into profiles/)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-pr}
export TMPDIR=/tmp
bash tools/pmc_bench.sh $TAG > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 1; }
cp gpurun_out/pmcb_$TAG/traffic.json profiles/r01/pmc_traffic.json
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cp profiles/r01/pmc_traffic.json gpurun_out/${TAG}_pmc_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
f=$(find gpurun_out/prof_$TAG -name "*kernel_trace.csv" | head -1)
python tools/trace_decode.py $f > gpurun_out/${TAG}_trace.txt 2>&1
cp $(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1) gpurun_out/${TAG}_kernel_stats.csv
tail -1 gpurun_out/${TAG}_bench.json
