#!/bin/bash
# int8 GEMM op tests + QKV / MLP-1 timing (default form), MFMA on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_6_ops.py -k "gemm_i8 or gelu or repeat" > gpurun_out/i8_epi_tests.log 2>&1 || { tail -30 gpurun_out/i8_epi_tests.log; exit 1; }
tail -1 gpurun_out/i8_epi_tests.log
for NM in 0 1; do
  echo "== NOMFMA=$NM $(ICAP_I8_NOMFMA=$NM timeout -k 10 120 python tools/gemm_shapes.py 20 2>/dev/null | grep -E "qkv|mlp0" | sed 's/.*| i8x2/i8x2/' | tr '\n' ' ')" || exit 1
done
