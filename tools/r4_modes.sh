#!/bin/bash
# Round 4: the other bench modes on the final tree (SCST reward step at the config-5 shape, beam 5, Grid beam 5).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; mkdir -p $O
for m in "scst --batch 128" "beam" "beam --model grid"; do
  tag=$(echo $m | tr ' -' '__')
  timeout -k 10 300 python bench.py --no-cpu-baseline --mode $m > $O/modes_$tag.json 2> $O/modes_$tag.err || { tail -5 $O/modes_$tag.err; exit 1; }
  tail -1 $O/modes_$tag.json | cut -c1-220
done
