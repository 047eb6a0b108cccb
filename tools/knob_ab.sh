#!/bin/bash
# A/B of one tools-build knob: GPU tests (TESTS, default the parity + op suites) with KNOB=VAL, then the headline
# bench alternating the default and VAL.  usage: KNOB=ICAP_X VAL=2 [TESTS="..."] bash tools/knob_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
timeout -k 10 400 python -m image_caption_amd.build --tools > gpurun_out/r2/ab_build.log 2>&1 || { tail -5 gpurun_out/r2/ab_build.log; exit 1; }
env $KNOB=$VAL timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_1_parity.py tests/test_gpu_6_ops.py} -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/ab_tests.log 2>&1 || { tail -30 gpurun_out/r2/ab_tests.log; exit 1; }
tail -1 gpurun_out/r2/ab_tests.log
for v in default $VAL default $VAL; do
  echo "== $KNOB=$v"
  if [ $v = default ]; then E=""; else E="$KNOB=$v"; fi
  env $E timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>gpurun_out/r2/ab_bench.err | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
  grep -E "enc_attention" gpurun_out/r2/ab_bench.err | head -2
done
