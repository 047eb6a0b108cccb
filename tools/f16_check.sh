#!/bin/bash
# fp16 encoder check: fp16 op tests + engine parity in f16, bench f16 vs i8x2, kernel stats of the f16 bench.
# usage: bash tools/f16_check.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-x}
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_6_ops.py tests/test_gpu_2_engine.py tests/test_gpu_1_parity.py -m gpu -x -q \
  -k "f16" --timeout 200 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -40 $O/${T}_tests.log; exit 1; }
tail -2 $O/${T}_tests.log
for p in f16 i8x2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --precision $p > $O/${T}_$p.json 2> $O/${T}_$p.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$T -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --precision f16 > $O/prof_$T.log 2>&1 || exit 1
f=$(find $O/prof_$T -name "*kernel_stats.csv" | head -1)
head -25 $f | cut -d, -f1-8
