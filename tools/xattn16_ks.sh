#!/bin/bash
# fp16 cross-attention key split (ICAP_XATTN16_KS=2, tools build): decode/parity GPU tests with it on, then the
# headline bench with and without it.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 400 python -m image_caption_amd.build --tools > gpurun_out/r2/ks_build.log 2>&1 || { tail -5 gpurun_out/r2/ks_build.log; exit 1; }
ICAP_XATTN16_KS=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py tests/test_gpu_0_workloads.py tests/test_gpu_6_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/ks_tests.log 2>&1 || { tail -30 gpurun_out/r2/ks_tests.log; exit 1; }
tail -1 gpurun_out/r2/ks_tests.log
for ks in 1 2 1 2; do
  echo "== ICAP_XATTN16_KS=$ks"
  ICAP_XATTN16_KS=$ks timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
