set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/base_tests.log 2>&1 || { tail -30 gpurun_out/r4/base_tests.log; exit 1; }
tail -2 gpurun_out/r4/base_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4/base_vit.json 2> gpurun_out/r4/base_vit.err || { tail -20 gpurun_out/r4/base_vit.err; exit 1; }
cat gpurun_out/r4/base_vit.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/base_prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4/base_prof.log 2>&1 || exit 1
f=$(find gpurun_out/r4/base_prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_decode.py $f > gpurun_out/r4/base_decode_trace.txt 2>&1
cp $f gpurun_out/r4/base_kernel_trace.csv
cat gpurun_out/r4/base_decode_trace.txt
