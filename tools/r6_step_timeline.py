"""Round 6: the timeline of one bench step outside the decode graph - every dispatch of the last timed step that is
not a decode-graph kernel (encoder kernels, copies, torch ops), with its duration and the gap before it, plus the
decode region's total - from a rocprofv3 kernel trace of `bench.py --steps 2 --warmup 1`.  Measurement tool.
usage: python tools/r6_step_timeline.py KERNEL_TRACE.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
DEC = ("dec_sa", "dec_chain", "dec_ffn", "cross_attn", "residual_layernorm", "head_kernel", "fill_", "embed_kernel")
# the last step: from the last im2col (the encoder's first kernel) to the end
starts = [i for i, r in enumerate(rows) if "im2col" in r["Kernel_Name"]]
seg = rows[starts[-1]:]
prev_end = None
dec_n = dec_t = 0
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    prev_end = e
    if any(k in name for k in DEC):
        dec_n += 1
        dec_t += (e - s) / 1e3
        continue
    print(f"{(s - t0) / 1e3:10.1f} us  {name:60s} {(e - s) / 1e3:8.2f} us  gap {gap:7.2f}")
print(f"decode-graph dispatches {dec_n}, busy {dec_t:.1f} us; step span {(prev_end - t0) / 1e3:.1f} us")
