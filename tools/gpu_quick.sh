#!/bin/bash
# One GPU round-trip for a subset: pytest -m gpu -k "$1" (file list in $2), then optional bench args in $3.
# usage: bash tools/gpu_quick.sh KEXPR "TEST FILES" "BENCH ARGS"
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest ${2:-tests} -m gpu -x -q -k "$1" > gpurun_out/tq.log 2>&1 || { tail -40 gpurun_out/tq.log; exit 1; }
tail -3 gpurun_out/tq.log
if [ -n "$3" ]; then
  timeout -k 10 400 python bench.py $3 > gpurun_out/bq.log 2>&1 || { tail -30 gpurun_out/bq.log; exit 1; }
  tail -1 gpurun_out/bq.log
fi
