"""Concurrency in a rocprofv3 kernel trace: over the decode region (first to last dec_self_attn),
the sum of kernel durations vs the wall span (>1 means kernels overlapped), and how many kernels
started while another was still running.  usage: python tools/trace_overlap.py run_kernel_trace.csv"""
import csv
import sys

with open(sys.argv[1]) as f:
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f)),
                  key=lambda r: r[1])
idx = [i for i, r in enumerate(rows) if "dec_self_attn" in r[0]]
# last decode call: from the last head-less gap... take the final 60% of self-attn launches
seg = rows[idx[len(idx) // 2]: idx[-1] + 1]
busy = sum(e - s for _, s, e in seg)
wall = seg[-1][2] - seg[0][1]
over, run_end = 0, 0
for _, s, e in seg:
    if s < run_end:
        over += 1
    run_end = max(run_end, e)
print(f"kernels {len(seg)}  sum(dur) {busy / 1e3:.1f} us  wall {wall / 1e3:.1f} us  ratio {busy / wall:.2f}  "
      f"started-while-busy {over}")
