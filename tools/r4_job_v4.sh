set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_gpu_6_ops.py tests/test_gpu_0_workloads.py tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py tests/test_scst.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r4/v4_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r4/v4_tests.log | head -20; tail -3 gpurun_out/r4/v4_tests.log; exit 1; }
tail -1 gpurun_out/r4/v4_tests.log; grep "greedy vs oracle" gpurun_out/r4/v4_tests.log
PYTHONPATH=. timeout -k 10 120 python tools/attn_repeat.py 256 197 12 2>&1 | grep -v amdgpu.ids || exit 1
for i in 1 2; do PYTHONPATH=. timeout -k 10 120 python tools/attn_time.py "product" 2>&1 | grep -v amdgpu.ids || exit 1; done
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4/v4_vit.json 2> gpurun_out/r4/v4_vit.err || { tail -5 gpurun_out/r4/v4_vit.err; exit 1; }
python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print("vit", d["value"], d["ms_per_step"], "enc", p["encoder"]["ms_per_step"], "dec", p["decode"]["ms_per_step"])' gpurun_out/r4/v4_vit.json; done
timeout -k 10 300 python bench.py --fp32-weights --no-cpu-baseline > gpurun_out/r4/v4_fp32w.json 2> gpurun_out/r4/v4_fp32w.err || { tail -5 gpurun_out/r4/v4_fp32w.err; exit 1; }
tail -1 gpurun_out/r4/v4_fp32w.json | cut -c1-250
timeout -k 10 300 python bench.py --fp32-weights --mode beam --no-cpu-baseline > gpurun_out/r4/v4_fp32w_beam.json 2> gpurun_out/r4/v4_fp32w_beam.err || { tail -5 gpurun_out/r4/v4_fp32w_beam.err; exit 1; }
tail -1 gpurun_out/r4/v4_fp32w_beam.json | cut -c1-250
timeout -k 10 300 python bench.py --mode beam --no-cpu-baseline > gpurun_out/r4/v4_beam.json 2> gpurun_out/r4/v4_beam.err || { tail -5 gpurun_out/r4/v4_beam.err; exit 1; }
tail -1 gpurun_out/r4/v4_beam.json | cut -c1-250
bash tools/r4_trace1.sh v4 'ICAP_DEC_BRANCHES=1'
