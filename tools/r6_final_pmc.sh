#!/bin/bash
# Round 6: the fp16 plane past 2 GiB test, then the PMC traffic passes of the final tree (tools/pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_6_ops.py -x -q --timeout 150 --timeout-method thread -k "past_2gib" > $O/big_test.log 2>&1 || { tail -30 $O/big_test.log; exit 1; }
tail -1 $O/big_test.log
ROUND=r6 bash tools/pmc.sh
