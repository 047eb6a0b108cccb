#!/bin/bash
# Persistent residual fp16 GEMMs (ICAP_F16_PRES=1, tools lib): op tests, the four ViT shapes, then the headline A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r2
mkdir -p $O
ICAP_F16_PRES=1 timeout -k 10 200 python -c "
import sys
from image_caption_amd import _lib
_lib.load('tools/libicap_tools.so')
import pytest
sys.exit(pytest.main(['tests/test_gpu_6_ops.py','-m','gpu','-x','-q','-k','gemm_f16','-p','no:cacheprovider']))
" > $O/pres_ops.log 2>&1 || { tail -30 $O/pres_ops.log; exit 1; }
tail -1 $O/pres_ops.log
for v in 0 1; do
  echo "== ICAP_F16_PRES=$v"
  ICAP_F16_PRES=$v timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done
rm -f tools/libicap_tools.so
KNOB=ICAP_F16_PRES VAL=1 bash tools/knob_ab.sh
