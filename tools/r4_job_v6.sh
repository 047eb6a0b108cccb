set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_gpu_6_ops.py tests/test_gpu_0_workloads.py tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py tests/test_scst.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r4/v6_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r4/v6_tests.log | head -20; tail -3 gpurun_out/r4/v6_tests.log; exit 1; }
tail -1 gpurun_out/r4/v6_tests.log; grep "greedy vs oracle" gpurun_out/r4/v6_tests.log
echo "== xattn"; timeout -k 10 120 python tools/xattn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4/v6_vit.json 2> gpurun_out/r4/v6_vit.err || { tail -5 gpurun_out/r4/v6_vit.err; exit 1; }
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print("vit", d["value"], d["ms_per_step"], "enc", p["encoder"]["ms_per_step"], "dec", p["decode"]["ms_per_step"])' gpurun_out/r4/v6_vit.json; done
