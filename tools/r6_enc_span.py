"""Round 6: the encoder of the last bench step from a rocprofv3 kernel trace - its span (first encoder kernel start to
the projection GEMM's end), the kernels' summed durations, and the gaps; both streams' kernels counted (the two-stream
encoder).  Measurement tool.  usage: python tools/r6_enc_span.py KERNEL_TRACE.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "im2col" in r["Kernel_Name"]]
last = starts[-1]
heads = [i for i in range(last) if "head_kernel" in rows[i]["Kernel_Name"]]  # the previous step's decode ends here
first = next(i for i in range(heads[-1] + 1 if heads else 0, len(rows)) if "im2col" in rows[i]["Kernel_Name"])
seg = []
for r in rows[first:]:
    n = r["Kernel_Name"]
    if any(k in n for k in ("dec_sa", "dec_chain", "dec_ffn", "cross_attn", "residual_layernorm", "head_kernel")):
        break
    seg.append(r)
t0 = int(seg[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in seg)
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
# union of kernel intervals (time with at least one encoder kernel running)
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
union, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce:
        union += ce - cs
        cs, ce = s, e
    else:
        ce = max(ce, e)
union += ce - cs
print(f"encoder kernels {len(seg)}: span {(t1 - t0) / 1e3:.1f} us, summed durations {busy / 1e3:.1f} us, "
      f"covered {union / 1e3:.1f} us, idle {(t1 - t0 - union) / 1e3:.1f} us")
for r in seg[:6]:
    print(f"  {(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} us {r['Kernel_Name'][:60]} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:.1f} us")
