#!/bin/bash
# Round-3 decode probe: headline bench at 1 / 2 / 3 decode chains (tools build: ICAP_DEC_MIN_ROWS), and a rocprofv3
# kernel trace of the 1-chain decode (no inter-chain contention) with per-kernel averages.
# usage: bash tools/r3_decode_probe.sh   (outputs under gpurun_out/r3/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 400 python -m image_caption_amd.build --tools > $O/dp_build.log 2>&1 || { tail -5 $O/dp_build.log; exit 1; }
for c in 1 2 3; do
  echo "== chains=$c"
  ICAP_DEC_MIN_ROWS=16 timeout -k 10 150 python bench.py --no-cpu-baseline --steps 10 --warmup 2 --decode-chains $c 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])' || exit 1
done
for c in 1 3; do
  ICAP_DEC_MIN_ROWS=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/dp_prof$c -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --decode-chains $c > $O/dp_prof$c.log 2>&1 || exit 1
  f=$(find $O/dp_prof$c -name "*kernel_trace.csv" | head -1)
  echo "== trace chains=$c"
  python3 tools/trace_decode.py $f | head -24
done
