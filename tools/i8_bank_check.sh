#!/bin/bash
# int8 GEMM after the LDS swizzle change: op tests under both tile forms, timing, bank conflicts.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for T in 128 256; do
  ICAP_I8_TILE=$T timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_6_ops.py -k "gemm_i8" > gpurun_out/i8b_tests.log 2>&1 || { tail -30 gpurun_out/i8b_tests.log; exit 1; }
  echo "tile $T: $(tail -1 gpurun_out/i8b_tests.log)"
done
echo "== $(timeout -k 10 120 python tools/gemm_shapes.py 20 2>/dev/null | grep -E "qkv|mlp0" | sed 's/.*| i8x2/i8x2/' | tr '\n' ' ')" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/i8bank -o run -- python3 $R/tools/gemm_shapes.py 2 > $R/gpurun_out/i8bank.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/i8bank | grep -A 5 "gemm_i8"
