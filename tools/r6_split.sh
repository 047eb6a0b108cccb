#!/bin/bash
# (Historical: the variant this script measured was removed from the sources after the measurement - see DESIGN.md;
# build it from the commit named there to rerun.)
# Round 6: the split last query tile of the persistent encoder attention - op and workload parity on the tree's library,
# then kernel stats and bench lines against the unsplit form (tools/ab/libicap_nosplit.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_6_ops.py tests/test_gpu_0_workloads.py tests/test_gpu_2_engine.py -x -q -s --timeout 120 --timeout-method thread -k "attention or config2 or pipeline or repeat" > $O/split_tests.log 2>&1; rc=$?
grep -E "passed|failed|greedy vs oracle|Error" $O/split_tests.log | tail -8
[ $rc -eq 0 ] || { tail -30 $O/split_tests.log; exit 1; }
bash tools/r6_kstats.sh sp image_caption_amd/libicap.so tools/ab/libicap_nosplit.so 2>&1 | grep -E "==|enc_attention|gemm_f16p"
ROUND=r6 bash tools/ab_libs.sh split 3 image_caption_amd/libicap.so tools/ab/libicap_nosplit.so
