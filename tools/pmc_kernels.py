"""Per-kernel mean of every counter per launch from rocprofv3 --pmc passes
(<root>/p*/run_counter_collection.csv) -> a text table on stdout."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k[:110])
    for c, v in sorted(d.items()):
        print(f"    {c:28s} {sum(v) / len(v):16.1f}  ({len(v)} launches)")
