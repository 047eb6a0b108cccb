#!/bin/bash
# 16-byte output stores of the fp16 encoder attention: the whole GPU suite, the headline bench twice, and a
# rocprofv3 --stats pass of the bench (enc_attention_pipe_kernel average).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/ea16w_tests.log 2>&1 || { tail -30 gpurun_out/r2/ea16w_tests.log; exit 1; }
tail -1 gpurun_out/r2/ea16w_tests.log
for i in 1 2; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof_ea -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2/prof_ea.log 2>&1 || exit 1
grep -h "enc_attention\|gemm_f16p" $(find gpurun_out/r2/prof_ea -name "*kernel_stats.csv") | cut -c1-200
