"""GPU idle gaps between consecutive kernels of a rocprofv3 kernel trace (one queue):
total busy vs wall time over the last N steps, and the kernels that follow the largest
gaps (where the GPU waited for the host).  usage: trace_gaps.py run_kernel_trace.csv [marker]"""
import csv, sys
from collections import defaultdict
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1]))))
marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
ends = [i for i, r in enumerate(rows) if marker in r[2]]
if len(ends) >= 3:   # the last two steps: from after the 3rd-last marker to the last
    rows = rows[ends[-3] + 1:ends[-1] + 1]
busy = sum(e - s for s, e, _ in rows)
wall = rows[-1][1] - rows[0][0]
gaps = defaultdict(float)
cnt = defaultdict(int)
for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
    g = s1 - e0
    if g > 2000:
        k = n1.split("(")[0].replace("void ", "")[:60]
        gaps[k] += g / 1e3
        cnt[k] += 1
print(f"steps in window: 2  wall {wall/2e6:.3f} ms/step  busy {busy/2e6:.3f} ms/step  idle {(wall-busy)/2e6:.3f} ms/step")
for k, v in sorted(gaps.items(), key=lambda x: -x[1])[:15]:
    print(f"  {v/2:8.1f} us/step idle before {cnt[k]/2:5.1f}x  {k}")
