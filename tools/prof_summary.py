"""Summarize a rocprofv3 --stats kernel_stats.csv: top kernels, % of time, per-step ms."""
import csv, sys
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    print("%6.2f%% %9.1f us avg %6d calls %8.3f ms/step  %s" % (100 * float(r['TotalDurationNs']) / tot, float(r['AverageNs']) / 1e3,
          int(r['Calls']), float(r['TotalDurationNs']) / 1e6 / steps, r['Name'][:90]))
print("total kernel ms per step: %.3f" % (tot / 1e6 / steps))
