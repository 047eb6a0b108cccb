set -o pipefail
for cfg in "ICAP_EAF_VAR=0" "ICAP_EAF_VAR=2" "ICAP_EAF_VAR=0" "ICAP_EAF_VAR=2" "ICAP_EAF_VAR=2 ICAP_EAF_ABL=1" "ICAP_EAF_VAR=2 ICAP_EAF_ABL=2"; do env $cfg PYTHONPATH=. timeout -k 10 120 python tools/attn_time.py "$cfg" 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/r4_tools_pytest.sh v2p 'ICAP_EAF_VAR=2' '-k enc_attention' tests/test_gpu_6_ops.py || exit 1
mkdir -p gpurun_out/r4
timeout -k 10 300 python bench.py --fp32-weights --no-cpu-baseline > gpurun_out/r4/v2_fp32w.json 2> gpurun_out/r4/v2_fp32w.err || { tail -5 gpurun_out/r4/v2_fp32w.err; exit 1; }
tail -1 gpurun_out/r4/v2_fp32w.json | cut -c1-400
timeout -k 10 300 python bench.py --fp32-weights --mode beam --no-cpu-baseline > gpurun_out/r4/v2_fp32w_beam.json 2> gpurun_out/r4/v2_fp32w_beam.err || { tail -5 gpurun_out/r4/v2_fp32w_beam.err; exit 1; }
tail -1 gpurun_out/r4/v2_fp32w_beam.json | cut -c1-400
timeout -k 10 300 python bench.py --mode beam --no-cpu-baseline > gpurun_out/r4/v2_beam.json 2> gpurun_out/r4/v2_beam.err || { tail -5 gpurun_out/r4/v2_beam.err; exit 1; }
tail -1 gpurun_out/r4/v2_beam.json | cut -c1-400
