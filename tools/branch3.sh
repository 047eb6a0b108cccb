#!/bin/bash
# decode chains per batch: 2 (default) vs 3 (86/85/85 rows) vs 4, headline bench; engine tests under 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
ICAP_DEC_BRANCHES=3 ICAP_DEC_MIN_ROWS=80 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_2_engine.py > gpurun_out/br3_tests.log 2>&1 || { tail -30 gpurun_out/br3_tests.log; exit 1; }
tail -1 gpurun_out/br3_tests.log
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 3 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
for V in "ICAP_DEC_BRANCHES=2" "ICAP_DEC_BRANCHES=3 ICAP_DEC_MIN_ROWS=80" "ICAP_DEC_BRANCHES=4 ICAP_DEC_MIN_ROWS=64" "ICAP_DEC_BRANCHES=2"; do
  echo "== $V $(env $V bash -c "$(declare -f run); run")" || exit 1
done
