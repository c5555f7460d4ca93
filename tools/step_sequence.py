"""Kernel sequence of the last whole training step in a rocprofv3 kernel trace, with
consecutive repeats collapsed (name x count, total us): shows where the small torch
kernels (fills, copies) sit between the library's launches.
usage: step_sequence.py run_kernel_trace.csv [marker]"""
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
marker = sys.argv[2] if len(sys.argv) > 2 else "adam_kernel"
ends = [i for i, r in enumerate(rows) if marker in r[2]]
if len(ends) >= 2:
    rows = rows[ends[-2] + 1:ends[-1] + 1]
out = []
for s, e, n in rows:
    k = n.split("(")[0].replace("void ", "")[:70]
    if out and out[-1][0] == k:
        out[-1][1] += 1
        out[-1][2] += (e - s) / 1e3
    else:
        out.append([k, 1, (e - s) / 1e3])
for k, c, t in out:
    print(f"{c:4d} x {t:9.1f} us  {k}")
