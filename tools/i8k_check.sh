#!/bin/bash
# Block-scaled i8x2 MLP pair: op test, i8x2 parity tests, A/B bench (ICAP_I8_MLP2=0 vs 1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_6_ops.py -x -v --timeout 120 --timeout-method thread -k "block_scaled or gemm_i8" > gpurun_out/i8k_ops.log 2>&1 || { tail -40 gpurun_out/i8k_ops.log; exit 1; }
tail -2 gpurun_out/i8k_ops.log
ICAP_I8_MLP2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py -x -q --timeout 120 --timeout-method thread -k i8x2 > gpurun_out/i8k_parity.log 2>&1 || { tail -40 gpurun_out/i8k_parity.log; exit 1; }
tail -2 gpurun_out/i8k_parity.log
for r in 1 2; do
timeout -k 10 200 env ICAP_I8_MLP2=0 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/i8k_off_$r.json 2>gpurun_out/i8k_off.err || exit 1
timeout -k 10 200 env ICAP_I8_MLP2=1 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/i8k_on_$r.json 2>gpurun_out/i8k_on.err || exit 1
done
for f in gpurun_out/i8k_off_*.json gpurun_out/i8k_on_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
