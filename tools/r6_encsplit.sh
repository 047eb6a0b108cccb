#!/bin/bash
# Round 6: the f16 ViT encoder as two half batches on two streams - the whole GPU suite on the tree's library, bench
# lines against the one-stream encoder (tools/abx/libicap_nosplit.so, -DICAP_ENC_SPLIT=0), then kernel stats of both.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/encsplit_tests.log 2>&1; rc=$?
grep -E "passed|failed|greedy vs oracle|outliers|Error" $O/encsplit_tests.log | tail -10
[ $rc -eq 0 ] || { tail -30 $O/encsplit_tests.log; exit 1; }
ROUND=r6 bash tools/ab_libs.sh encsplit 3 image_caption_amd/libicap.so tools/abx/libicap_nosplit.so || exit 1
bash tools/r6_kstats.sh es image_caption_amd/libicap.so tools/abx/libicap_nosplit.so 2>&1 | grep -E "==|enc_attention|gemm_f16p|layernorm_kernel"
