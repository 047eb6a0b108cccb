#!/bin/bash
# fp16 GEMM forms on the ViT shapes (tools/libicap_tools.so: ICAP_F16_GEMM 0 = 128x256 32-deep 2 blocks/CU,
# 3 / 4 = 128x256 64-deep 2 / 3 stages, 5 = 256x256 64-deep), each form's op test first.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2
mkdir -p $O
for f in ${FORMS:-0 3 4 5}; do
  ICAP_F16_GEMM=$f timeout -k 10 200 python -c "
import sys
from image_caption_amd import _lib
_lib.load('tools/libicap_tools.so')
import pytest
sys.exit(pytest.main(['tests/test_gpu_6_ops.py','-m','gpu','-x','-q','-k','gemm_f16','-p','no:cacheprovider']))
" > $O/f16form_ops$f.log 2>&1 || { tail -30 $O/f16form_ops$f.log; exit 1; }
  echo "== ICAP_F16_GEMM=$f ($(tail -1 $O/f16form_ops$f.log))"
  ICAP_F16_GEMM=$f timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done
