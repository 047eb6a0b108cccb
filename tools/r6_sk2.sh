#!/bin/bash
# (Historical: the variant this script measured was removed from the sources after the measurement - see DESIGN.md;
# build it from the commit named there to rerun.)
# Round 6: where stream-K's time goes - per-launch encoder GEMM durations of one bench step (kernel trace, first ViT
# layer of the last step) for stream-K on / compiled-in but off / not compiled, then bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
for L in image_caption_amd/libicap.so tools/ab/libicap_skoff.so tools/ab/libicap_nosk.so; do
  n=$(basename $L .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/sk2_$n -o run -- python3 -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('$L')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '2', '--warmup', '1']
runpy.run_path('bench.py', run_name='__main__')
" > $O/sk2_$n.log 2>&1 || { tail -5 $O/sk2_$n.log; exit 1; }
  f=$(find $O/sk2_$n -name "*kernel_trace.csv" | head -1)
  echo "== $n"
  python3 tools/r6_step_timeline.py $f > $O/sk2_${n}_timeline.txt
  grep -E "gemm_f16p|enc_attention|layernorm_kernel" $O/sk2_${n}_timeline.txt | head -8
  find $O/sk2_$n -name "*.csv" -delete
done
ROUND=r6 bash tools/ab_libs.sh sk2 2 image_caption_amd/libicap.so tools/ab/libicap_skoff.so tools/ab/libicap_nosk.so
