#!/bin/bash
# Round 6: the other bench modes on the final tree (SCST reward step, beam 5, fp32-checkpoint decoder weights).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
run() { n=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }; python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["metric"][:40], d["value"], d["unit"], d["ms_per_step"])' $O/bench_$n.json $n; }
run scst_b128 --mode scst --batch 128
run beam5_vit --mode beam
run beam5_grid --mode beam --model grid
run vit_fp32w --fp32-weights
run vit_fp32w_beam5 --fp32-weights --mode beam
# (pipelined greedy is the default since the end of round 6: the other precisions through the pipeline, and sequential)
[ -n "$R6_MODES_ALL" ] && { run vit_bf16x2 --precision bf16x2; run vit_i8x2 --precision i8x2; run vit_seq_fp32w --fp32-weights --sequential; run grid_seq --model grid --sequential; }
