#!/bin/bash
# int8 GEMM tile forms: op parity tests of the 128 x 256 one-block-per-CU form (ICAP_I8_TILE=256;
# the default 128 x 128 two-blocks-per-CU form runs in the normal suite), then QKV / MLP-1 timing
# of both, MFMA on / off (ICAP_I8_NOMFMA=1: staging + epilogue only).
set -o pipefail
cd $GRAFT_REPO_ROOT
ICAP_I8_TILE=256 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_6_ops.py -k "gemm_i8" > gpurun_out/i8_tile_tests.log 2>&1 || { tail -30 gpurun_out/i8_tile_tests.log; exit 1; }
tail -2 gpurun_out/i8_tile_tests.log
for V in "ICAP_I8_TILE=128" "ICAP_I8_TILE=256"; do for NM in 0 1; do
  echo "== $V NOMFMA=$NM $(env $V ICAP_I8_NOMFMA=$NM timeout -k 10 120 python tools/gemm_shapes.py 20 2>/dev/null | grep -E "qkv|mlp0" | sed 's/.*| i8x2/i8x2/' | tr '\n' ' ')" || exit 1
done; done
