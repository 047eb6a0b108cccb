#!/bin/bash
# Round 6: the product sources without the rejected variants (stream-K, LayerNorm folds, attention split) - the whole
# GPU suite, then bench lines against the library built from the tree before the removal (tools/abx/libicap_base.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/clean_tests.log 2>&1; rc=$?
grep -E "passed|failed|greedy vs oracle|outliers|Error" $O/clean_tests.log | tail -10
[ $rc -eq 0 ] || { tail -30 $O/clean_tests.log; exit 1; }
ROUND=r6 bash tools/ab_libs.sh clean 3 image_caption_amd/libicap.so tools/abx/libicap_base.so
