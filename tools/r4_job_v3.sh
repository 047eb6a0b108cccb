set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 200 python -u -m pytest tests/test_gpu_6_ops.py -k "enc_attention or full_chip" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/v3_tests.log 2>&1 || { tail -30 gpurun_out/r4/v3_tests.log; exit 1; }
tail -1 gpurun_out/r4/v3_tests.log
for i in 1 2; do PYTHONPATH=. timeout -k 10 120 python tools/attn_time.py "product" 2>&1 | grep -v amdgpu.ids || exit 1; done
PYTHONPATH=. ICAP_ENC_ATTN16_FULL=1 timeout -k 10 120 python tools/attn_repeat.py 256 197 12 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r4/v3_vit.json 2> gpurun_out/r4/v3_vit.err || { tail -5 gpurun_out/r4/v3_vit.err; exit 1; }
tail -1 gpurun_out/r4/v3_vit.json | cut -c1-300
timeout -k 10 300 python bench.py --fp32-weights --no-cpu-baseline > gpurun_out/r4/v3_fp32w.json 2> gpurun_out/r4/v3_fp32w.err || { tail -5 gpurun_out/r4/v3_fp32w.err; exit 1; }
tail -1 gpurun_out/r4/v3_fp32w.json | cut -c1-300
timeout -k 10 300 python bench.py --fp32-weights --mode beam --no-cpu-baseline > gpurun_out/r4/v3_fp32w_beam.json 2> gpurun_out/r4/v3_fp32w_beam.err || { tail -5 gpurun_out/r4/v3_fp32w_beam.err; exit 1; }
tail -1 gpurun_out/r4/v3_fp32w_beam.json | cut -c1-300
timeout -k 10 300 python bench.py --mode beam --no-cpu-baseline > gpurun_out/r4/v3_beam.json 2> gpurun_out/r4/v3_beam.err || { tail -5 gpurun_out/r4/v3_beam.err; exit 1; }
tail -1 gpurun_out/r4/v3_beam.json | cut -c1-300
