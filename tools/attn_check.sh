#!/bin/bash
# encoder attention: op tests (incl. the full-chip bitwise repeat), kernel time on the ViT encoder, bank conflicts.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_6_ops.py -k "attention or repeat" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
bash tools/attn_ab.sh "X=1" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/apmc_bc -o run -- python3 $R/tools/encode_grid.py 2 256 vit > $R/gpurun_out/apmc_bc.log 2>&1 || exit 1
cd $R && python3 tools/pmc_summary.py gpurun_out/apmc_bc | grep -A 5 "enc_attention_pipe"
