#!/bin/bash
# Round 6: the pipeline's attention budget (icap_set_encoder_attention_cus) - pipeline / engine tests, then alternating
# bench lines: default (GEMMs 160, attention 128 CUs), attention at the GEMMs' budget (0), attention 96.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_2_engine.py tests/test_host.py -x -q --timeout 200 --timeout-method thread > $O/pattn_tests.log 2>&1 || { tail -20 $O/pattn_tests.log; exit 1; }
tail -1 $O/pattn_tests.log
R6_PV_ROUNDS=3 R6_PV="default:X=1:;attn_gemm_budget:ICAP_PIPE_ENC_ATTN_CUS=0:;attn96:ICAP_PIPE_ENC_ATTN_CUS=96:" bash tools/r6_pipe_var.sh
cp $O/pipe_var.txt $O/pipe_attn_ab.txt
