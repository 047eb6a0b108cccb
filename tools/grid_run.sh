set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "grid" > gpurun_out/t_grid.log 2>&1 || { tail -40 gpurun_out/t_grid.log; exit 1; }
tail -3 gpurun_out/t_grid.log
timeout -k 10 300 python bench.py --model grid --steps 5 --warmup 2 > gpurun_out/bg.log 2>&1 || { tail -30 gpurun_out/bg.log; exit 1; }
tail -1 gpurun_out/bg.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_grid -o run -- python3 $R/bench.py --model grid --steps 3 --warmup 1 > $R/gpurun_out/bgp.log 2>&1 || { tail -30 $R/gpurun_out/bgp.log; exit 1; }
find $R/gpurun_out/prof_grid -name "*kernel_stats.csv" | head -3
