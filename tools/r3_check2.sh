#!/bin/bash
# Round-3 check of the product build: the GPU suite as the driver runs it, smoke(), the headline bench line and the
# Grid bench line.  usage: bash tools/r3_check2.sh TAG   (outputs under gpurun_out/r3/)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-c}
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=25 > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log | cut -c1-80
timeout -k 10 300 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -20 $O/${T}_bench.err; exit 1; }
timeout -k 10 300 python bench.py --model grid > $O/${T}_bench_grid.json 2> $O/${T}_bench_grid.err || { tail -20 $O/${T}_bench_grid.err; exit 1; }
for f in $O/${T}_bench.json $O/${T}_bench_grid.json; do
  tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; p=r["phases"]; print(d["config"]["workload"][:20], d["value"], d["ms_per_step"], "enc", p["encoder"]["ms_per_step"], "dec", p["decode"]["ms_per_step"], r["kernel"], r["frac"])'
done
