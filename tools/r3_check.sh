#!/bin/bash
# Round-3 check: the GPU suite exactly as the driver runs it (plus per-test durations), smoke(), and the headline
# bench line.  usage: bash tools/r3_check.sh TAG   (outputs under gpurun_out/r3/)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-c}
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread --durations=25 > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -3 $O/${T}_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/${T}_smoke.log 2>&1 || { tail -20 $O/${T}_smoke.log; exit 1; }
tail -1 $O/${T}_smoke.log
timeout -k 10 300 python bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -20 $O/${T}_bench.err; exit 1; }
tail -1 $O/${T}_bench.json
