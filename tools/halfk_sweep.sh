#!/bin/bash
# 128x256 / 2-stage / 2-blocks-per-CU GEMM variant (ICAP_GEMM_TALL_MIN_K): parity with it forced on
# everywhere, trunk traces per threshold, ViT bench A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
ICAP_GEMM_TALL_MIN_K=1 timeout -k 10 600 python -m pytest tests/test_gpu_6_ops.py tests/test_gpu_1_parity.py -m gpu -x -q -k "gemm or grid or golden" > gpurun_out/hk_t.log 2>&1 || { tail -30 gpurun_out/hk_t.log; exit 1; }
tail -2 gpurun_out/hk_t.log
cd /tmp && export TMPDIR=/tmp
for H in 0 1 128 512; do
  ICAP_GEMM_TALL_MIN_K=$H timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/hk_$H -o run -- python3 $R/tools/encode_grid.py 2 256 > $R/gpurun_out/hk_$H.log 2>&1 || exit $?
  echo "H=$H $(tail -1 $R/gpurun_out/hk_$H.log)"
  python3 $R/tools/trunk_breakdown.py $R/gpurun_out/hk_$H/run_kernel_trace.csv > $R/gpurun_out/hk_$H.txt
done
cd $R
for H in 0 128 1024; do
  ICAP_GEMM_TALL_MIN_K=$H timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/hk_b$H.log 2>&1 || exit $?
  echo "vit H=$H $(tail -1 gpurun_out/hk_b$H.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
