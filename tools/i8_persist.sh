#!/bin/bash
# persistent vs per-tile i8 GEMM: op tests under both, shape timing, headline bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
for P in 1 0; do
  echo "== ICAP_I8_PERSIST=$P"
  ICAP_I8_PERSIST=$P timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py -m gpu -x -q -k "i8 or golden_per" --timeout 120 --timeout-method thread > gpurun_out/ip_t$P.log 2>&1; tail -2 gpurun_out/ip_t$P.log
  ICAP_I8_PERSIST=$P timeout -k 10 120 python tools/gemm_shapes.py 20 2>/dev/null | grep -E "qkv|mlp0" | sed 's/.*| i8x2/i8x2/' || exit 1
  ICAP_I8_PERSIST=$P timeout -k 10 150 python bench.py --no-cpu-baseline 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_us"])' || exit 1
done
