#!/bin/bash
# Full checkpoint: every GPU test, then the bench lines of every config (ViT headline, Grid, SCST, beam).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-rb}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_vit.json 2> gpurun_out/${TAG}_vit.err || { tail -20 gpurun_out/${TAG}_vit.err; exit 1; }
timeout -k 10 300 python bench.py --model grid --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_grid.json 2> gpurun_out/${TAG}_grid.err || exit 1
timeout -k 10 300 python bench.py --mode scst --batch 128 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_scst.json 2> gpurun_out/${TAG}_scst.err || exit 1
timeout -k 10 300 python bench.py --mode beam --beam 5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_beam.json 2> gpurun_out/${TAG}_beam.err || exit 1
for m in vit grid scst beam; do
  echo "$m $(tail -1 gpurun_out/${TAG}_$m.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms", d["roofline"]["kernel"], d["roofline"]["frac"])')"
done
