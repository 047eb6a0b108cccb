#!/bin/bash
# Round 5 batch: (1) the whole GPU suite on the tree's build (hi/lo fused decode, new config-2 fp32-weights test);
# (2) bench lines with --fp32-weights (greedy, beam 5) and the default, this tree against the round-4 library;
# (3) the Grid single-plane trunk variant through the config-3 checks; (4) the GEMM / attention variants' op tests
# and a same-box A/B of their bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5; mkdir -p $O
# (1)-(2) done: gpurun_out/r5/w2_*
timeout -k 10 300 python tools/r5_trunk_single.py tools/ab/libicap_t1.so > $O/t1_single.log 2>&1; tail -6 $O/t1_single.log
for L in lb prod nw7; do
  timeout -k 10 300 python tools/libtest.py tools/ab/libicap_$L.so tests/test_gpu_6_ops.py -k "gemm_f16 or enc_attention_f16 or full_chip" > $O/v_${L}_tests.log 2>&1 || { echo "variant $L FAILED"; tail -20 $O/v_${L}_tests.log; exit 1; }
  echo "variant $L: $(tail -1 $O/v_${L}_tests.log)"
done
bash tools/ab_libs.sh g2 3 image_caption_amd/libicap.so tools/ab/libicap_lb.so tools/ab/libicap_prod.so tools/ab/libicap_nw7.so tools/ab/libicap_base.so
