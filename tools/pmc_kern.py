"""Mean per-launch value of every collected counter for kernels whose name contains a filter.
usage: pmc_kern.py <dir with p*/...counter_collection.csv> [filter ...]"""
import csv, glob, os, sys
from collections import defaultdict
root, filt = sys.argv[1], sys.argv[2:] or ["ctn::"]
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if any(x in k for x in filt):
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k[:100])
    for c, v in sorted(d.items()):
        print("   %-28s %14.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
