#!/bin/bash
# 16-byte SO epilogue stores (default) against 8-byte (ABL 8): the whole GPU suite (product build), then (tools build) the four ViT shapes and
# the headline bench with ICAP_F16P_ABL=0 (16-B stores) / 8 (8-B stores) alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/f16w_tests.log 2>&1 || { tail -30 gpurun_out/r2/f16w_tests.log; exit 1; }
tail -1 gpurun_out/r2/f16w_tests.log
timeout -k 10 400 python -m image_caption_amd.build --tools > gpurun_out/r2/ab_build.log 2>&1 || { tail -5 gpurun_out/r2/ab_build.log; exit 1; }
for v in 0 8; do
  echo "== ICAP_F16P_ABL=$v"
  ICAP_F16P_ABL=$v timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids || exit 1
done
for v in 0 8 0 8; do
  echo "== ICAP_F16P_ABL=$v"
  ICAP_F16P_ABL=$v timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
