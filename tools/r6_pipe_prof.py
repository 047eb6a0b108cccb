"""Round 6: the live launch timing of the pipelined bench against the rocprofv3 kernel trace of the same command.
bench.py brackets ViT layers 0 and 6 of every timed encode (8 of the 48 gemm_f16p_kernel launches); the trace holds every
launch of the run: warmup encodes, the timed ones, the stop-rule check's sequential encode.  This picks the trace's
launches at the same positions (encodes warmup .. warmup + steps - 1, launches 0-3 and 24-27 of each) and prints their
average beside the trace-wide average and the live figure from the bench line in the log.
usage: python tools/r6_pipe_prof.py KERNEL_TRACE_CSV BENCH_LOG [STEPS WARMUP]"""
import csv
import json
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "gemm_f16p_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
steps, warmup = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (10, 3)
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
per = 48
n_enc = len(dur) // per
print(f"gemm_f16p_kernel launches in the trace: {len(dur)} ({n_enc} encodes of {per}), average {sum(dur) / len(dur):.2f} us")
for e in range(n_enc):
    d = dur[e * per:(e + 1) * per]
    role = "warmup" if e < warmup else ("timed" if e < warmup + steps else "stop-rule check (sequential)")
    print(f"  encode {e:2d} {role:30s} average {sum(d) / per:8.2f} us, layers 0 and 6 {sum(d[0:4] + d[24:28]) / 8:8.2f} us")
sel = [x for e in range(warmup, min(warmup + steps, n_enc)) for x in dur[e * per:e * per + 4] + dur[e * per + 24:e * per + 28]]
line = None
for ln in open(sys.argv[2]):
    if ln.startswith("{") and '"roofline"' in ln:
        line = json.loads(ln)
live = line["roofline"]["avg_launch_us"] if line else None
print(f"trace, the bench's timed launches (layers 0 and 6 of the {steps} timed encodes): {sum(sel) / len(sel):.2f} us over "
      f"{len(sel)} launches; the bench's live events in the same run: {live} us")
