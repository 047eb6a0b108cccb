#!/bin/bash
# Same-box A/B of two library builds: the encoder GEMM shapes (tools/gemm_f16.py) and the headline bench, alternating
# BASE (tools/libicap_base.so, copied over the product library for its bench runs) and the in-tree build.
# usage: bash tools/r3_lib_ab.sh [TESTS]   (TESTS: GPU test files run first on the in-tree build)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3; mkdir -p $O
if [ -n "$1" ]; then
  timeout -k 10 400 python -u -m pytest $1 -m gpu -x -q --timeout 120 --timeout-method thread > $O/ab_tests.log 2>&1 || { tail -30 $O/ab_tests.log; exit 1; }
  tail -1 $O/ab_tests.log
fi
cp image_caption_amd/libicap.so $O/libicap_new.so
for v in base new base new; do
  echo "== $v"
  GEMM_LIB=$O/libicap_$v.so; [ $v = base ] && GEMM_LIB=tools/libicap_base.so
  GEMM_LIB=$GEMM_LIB timeout -k 10 120 python tools/gemm_f16.py 20 2>&1 | grep -v amdgpu.ids || exit 1
  cp $GEMM_LIB image_caption_amd/libicap.so
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 $BENCH_ARGS 2>$O/ab_bench.err | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print("bench", d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"], d["roofline"]["avg_launch_us"])' || exit 1
done
cp $O/libicap_new.so image_caption_amd/libicap.so
