#!/bin/bash
# Split cross-attention (ICAP_XATTN_KS=2, default): every GPU test, then A/B bench against KS=1 (ViT greedy, beam).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xks_tests.log 2>&1 || { tail -40 gpurun_out/xks_tests.log; exit 1; }
tail -2 gpurun_out/xks_tests.log
for r in 1 2; do
for k in 1 2; do
timeout -k 10 200 env ICAP_XATTN_KS=$k python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/xks_vit_${k}_$r.json 2>gpurun_out/xks.err || exit 1
done
done
for k in 1 2; do
timeout -k 10 200 env ICAP_XATTN_KS=$k python bench.py --mode beam --beam 5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/xks_beam_${k}.json 2>gpurun_out/xks.err || exit 1
done
for f in gpurun_out/xks_vit_*.json gpurun_out/xks_beam_*.json; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/xksp -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/xksp.log 2>&1 || exit 1
f=$(find gpurun_out/xksp -name "*kernel_trace.csv" | head -1)
python tools/trace_decode.py $f > gpurun_out/xks_trace.txt 2>&1
head -16 gpurun_out/xks_trace.txt
