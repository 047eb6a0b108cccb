#!/bin/bash
# Grid tail attention (N = 49) after the swizzle change: op tests, Grid bench, bank conflicts.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_6_ops.py tests/test_gpu_1_parity.py -k "attention or repeat or grid" > gpurun_out/gattn_tests.log 2>&1 || { tail -30 gpurun_out/gattn_tests.log; exit 1; }
tail -1 gpurun_out/gattn_tests.log
timeout -k 10 300 python bench.py --model grid --steps 5 --warmup 2 --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("grid", d["value"], d["ms_per_step"])' || exit 1
BENCH_ARGS="--model grid" bash tools/bank_pmc.sh | grep enc_attention
