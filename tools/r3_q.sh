set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3/q_tests.log 2>&1 || { tail -30 gpurun_out/r3/q_tests.log; exit 1; }
tail -1 gpurun_out/r3/q_tests.log
bash tools/r3_lib_ab.sh && BENCH_ARGS="--model grid" bash tools/r3_lib_ab.sh 2>&1 | grep bench
