#!/bin/bash
# persistent fp16 GEMM: op + stress tests, the four ViT shapes, then the headline bench twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 300 python -u -m pytest tests/test_gpu_6_ops.py -m gpu -x -q -k "gemm_f16" --timeout 200 --timeout-method thread > gpurun_out/r2/f16p_tests.log 2>&1 || { tail -30 gpurun_out/r2/f16p_tests.log; exit 1; }
tail -1 gpurun_out/r2/f16p_tests.log
timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
