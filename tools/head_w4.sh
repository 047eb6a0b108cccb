#!/bin/bash
# decode head with the [D/4][V][4] fc_out image: the whole GPU suite (product build), then (tools build) the headline
# bench alternating ICAP_HEAD_W4=1 (default) / 0 and a rocprofv3 --stats pass for the head's launch time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2/hw4_tests.log 2>&1 || { tail -30 gpurun_out/r2/hw4_tests.log; exit 1; }
tail -1 gpurun_out/r2/hw4_tests.log
timeout -k 10 400 python -m image_caption_amd.build --tools > gpurun_out/r2/ab_build.log 2>&1 || { tail -5 gpurun_out/r2/ab_build.log; exit 1; }
for v in 1 0 1 0; do
  echo "== ICAP_HEAD_W4=$v"
  ICAP_HEAD_W4=$v timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
for v in 1 0; do
  ICAP_HEAD_W4=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof_hw4_$v -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r2/prof_hw4_$v.log 2>&1 || exit 1
  echo "W4=$v: $(grep -h '"(anonymous namespace)::head_kernel' $(find gpurun_out/r2/prof_hw4_$v -name '*kernel_stats.csv') | cut -c1-120)"
done
