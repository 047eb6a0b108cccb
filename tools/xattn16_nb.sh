#!/bin/bash
# fp16 cross-attention LDS ring depth (tools build, ICAP_XATTN16_NB 2 = default, 3, 4): decode parity / engine /
# SCST GPU tests with 3 and 4, then the headline bench alternating 2 / 3 / 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 400 python -m image_caption_amd.build --tools > gpurun_out/r2/ab_build.log 2>&1 || { tail -5 gpurun_out/r2/ab_build.log; exit 1; }
for v in 3 4; do
  ICAP_XATTN16_NB=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py tests/test_gpu_4_scst.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/nb_tests_$v.log 2>&1 || { tail -30 gpurun_out/r2/nb_tests_$v.log; exit 1; }
  echo "NB=$v: $(tail -1 gpurun_out/r2/nb_tests_$v.log)"
done
for v in 2 3 4 2 3 4; do
  echo "== ICAP_XATTN16_NB=$v"
  ICAP_XATTN16_NB=$v timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
