set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
for c in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --decode-chains $c > gpurun_out/r2/ch$c.json 2>/dev/null || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof_ch1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --decode-chains 1 > gpurun_out/r2/prof_ch1.log 2>&1 || exit 1
f=$(find gpurun_out/r2/prof_ch1 -name "*kernel_trace.csv" | head -1)
python tools/trace_decode.py $f > gpurun_out/r2/ch1_trace.txt 2>&1
