#!/bin/bash
# Round 4: the one-wave-per-SIMD fp16 GEMM (gemm_f16w_kernel, tools build ICAP_F16_GEMM 8 / 9 / 10) against the
# product form (0) on the ViT shapes, then its correctness on the op-level fp16 GEMM tests and the engine parity tests.
# usage: bash tools/r4_f16w.sh TAG [FORMS]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; mkdir -p $O
T=${1:-w}
FORMS=${2:-"0 8 9 10"}
for f in $FORMS; do
  echo "== ICAP_F16_GEMM=$f"
  ICAP_F16_GEMM=$f timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done | tee $O/${T}_gemm.txt
for f in ${CHECK:-8}; do
  ICAP_F16_GEMM=$f timeout -k 10 300 python -u -c "
import sys; sys.argv=['x']
import torch
from image_caption_amd import _lib
_lib.load('tools/libicap_tools.so')
import pytest
sys.exit(pytest.main(['tests/test_gpu_6_ops.py','tests/test_gpu_1_parity.py','tests/test_gpu_0_workloads.py','-m','gpu','-x','-q','-k','gemm_f16 or vit_golden or config2','-p','no:cacheprovider','--timeout','120','--timeout-method','thread']))
" > $O/${T}_ops$f.log 2>&1 || { tail -30 $O/${T}_ops$f.log; exit 1; }
  tail -3 $O/${T}_ops$f.log
done
# the key-split cross-attention (product build): op tests, then the decode parity tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_6_ops.py -m gpu -x -q -k cross_attn --timeout 120 --timeout-method thread > $O/${T}_xattn.log 2>&1 || { tail -30 $O/${T}_xattn.log; exit 1; }
tail -2 $O/${T}_xattn.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail -20 $O/${T}_bench.err; exit 1; }
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print("bench", d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' $O/${T}_bench.json
