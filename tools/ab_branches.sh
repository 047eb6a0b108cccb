#!/bin/bash
# A/B of the two-chain decode (ICAP_DEC_BRANCHES=2): parity tests with it on, then bench with 1 and 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
ICAP_DEC_BRANCHES=2 timeout -k 10 600 python -m pytest tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py -m gpu -x -q > gpurun_out/ab_t.log 2>&1 || { tail -30 gpurun_out/ab_t.log; exit 1; }
tail -2 gpurun_out/ab_t.log
for nb in 1 2; do
  ICAP_DEC_BRANCHES=$nb timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_b$nb.log 2>&1 || { tail -20 gpurun_out/ab_b$nb.log; exit 1; }
  echo "branches=$nb $(tail -1 gpurun_out/ab_b$nb.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
