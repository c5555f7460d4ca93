"""Summarize a rocprofv3 --stats kernel_stats.csv: top kernels, % of time, per-step ms.
bench.py's bandwidth calibration (ctn copy_stream_kernel, run once after the timed steps)
is listed apart and left out of the per-step figures."""
import csv, sys
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
calib = [r for r in rows if "copy_stream_kernel" in r['Name']]
rows = [r for r in rows if "copy_stream_kernel" not in r['Name']]
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    print("%6.2f%% %9.1f us avg %6d calls %8.3f ms/step  %s" % (100 * float(r['TotalDurationNs']) / tot, float(r['AverageNs']) / 1e3,
          int(r['Calls']), float(r['TotalDurationNs']) / 1e6 / steps, r['Name'][:90]))
print("total kernel ms per step: %.3f" % (tot / 1e6 / steps))
if calib:
    print("bench calibration copies (not per step): %d launches, %.1f ms" % (
        sum(int(r['Calls']) for r in calib), sum(float(r['TotalDurationNs']) for r in calib) / 1e6))
