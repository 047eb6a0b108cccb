#!/bin/bash
# (Historical: the variant this script measured was removed from the sources after the measurement - see DESIGN.md;
# build it from the commit named there to rerun.)
# Round 6: stream-K timing ablation - per-launch encoder GEMM durations (first ViT layer of a bench step) with the
# partial exchange removed (ICAP_SK_ABL=2: wrong sums, timing only) against stream-K and whole tiles.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
for L in tools/ab/libicap_skabl2.so image_caption_amd/libicap.so tools/ab/libicap_nosk.so; do
  n=$(basename $L .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/sk3_$n -o run -- python3 -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('$L')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '2', '--warmup', '1']
runpy.run_path('bench.py', run_name='__main__')
" > $O/sk3_$n.log 2>&1 || { tail -5 $O/sk3_$n.log; exit 1; }
  f=$(find $O/sk3_$n -name "*kernel_trace.csv" | head -1)
  echo "== $n"
  python3 tools/r6_step_timeline.py $f > $O/sk3_${n}_timeline.txt
  grep -E "gemm_f16p" $O/sk3_${n}_timeline.txt | head -8
  find $O/sk3_$n -name "*.csv" -delete
done
