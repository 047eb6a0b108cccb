#!/bin/bash
# fp16 GEMM forms on the ViT shapes (tools build), then the f16 op tests and bench (product build).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out/r2
mkdir -p $O
for f in 0 1 2; do
  echo "== ICAP_F16_GEMM=$f"
  ICAP_F16_GEMM=$f timeout -k 10 120 python tools/gemm_f16.py 20 || exit 1
done > $O/${T}_gemm.txt 2>&1
cat $O/${T}_gemm.txt
for f in 1 2; do
  ICAP_F16_GEMM=$f timeout -k 10 200 python -c "
import sys; sys.argv=['x']
import torch, os
from image_caption_amd import _lib
_lib.load('tools/libicap_tools.so')
import pytest
sys.exit(pytest.main(['tests/test_gpu_6_ops.py','-m','gpu','-x','-q','-k','gemm_f16','-p','no:cacheprovider']))
" > $O/${T}_ops$f.log 2>&1 || { tail -30 $O/${T}_ops$f.log; exit 1; }
  tail -1 $O/${T}_ops$f.log
done
timeout -k 10 200 python bench.py --no-cpu-baseline --precision f16 > $O/${T}_f16.json 2> $O/${T}_f16.err || exit 1
tail -4 $O/${T}_f16.err
cat $O/${T}_f16.json
