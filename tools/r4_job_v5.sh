set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_6_ops.py tests/test_gpu_0_workloads.py -k "enc_attention or full_chip or config2" -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r4/v5_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r4/v5_tests.log | head; tail -3 gpurun_out/r4/v5_tests.log; exit 1; }
tail -1 gpurun_out/r4/v5_tests.log; grep "greedy vs oracle" gpurun_out/r4/v5_tests.log
for shape in "256 197 12" "2 197 12"; do PYTHONPATH=. timeout -k 10 120 python tools/attn_repeat.py $shape 2>&1 | grep -v amdgpu.ids || exit 1; done
for i in 1 2; do PYTHONPATH=. timeout -k 10 120 python tools/attn_time.py "product" 2>&1 | grep -v amdgpu.ids || exit 1; done
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4/v5_vit.json 2> gpurun_out/r4/v5_vit.err || { tail -5 gpurun_out/r4/v5_vit.err; exit 1; }
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print("vit", d["value"], d["ms_per_step"], "enc", p["encoder"]["ms_per_step"], "dec", p["decode"]["ms_per_step"])' gpurun_out/r4/v5_vit.json; done
