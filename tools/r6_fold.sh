#!/bin/bash
# (Historical: the variant this script measured was removed from the sources after the measurement - see DESIGN.md;
# build it from the commit named there to rerun.)
# Round 6: the LayerNorm fold - the encoder / workload parity tests on the tree's library (fold on), then bench lines
# alternating fold on / off (tools/ab/libicap_nofold.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_0_workloads.py tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py -x -q -s --timeout 120 --timeout-method thread > $O/fold_tests.log 2>&1; rc=$?
grep -E "passed|failed|greedy vs oracle|outliers|Error" $O/fold_tests.log | tail -12
[ $rc -eq 0 ] || { tail -30 $O/fold_tests.log; exit 1; }
ROUND=r6 bash tools/ab_libs.sh fold 3 image_caption_amd/libicap.so tools/ab/libicap_nofold.so
