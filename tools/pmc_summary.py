"""Per-kernel mean of rocprofv3 --pmc counters over passes p1..pN (gpurun_out/pmc)."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
def short(n):
    n = n.replace("ctn::", "").replace("unsigned short", "bf16")
    return n[:70]
keys = sorted(vals, key=lambda k: -len(vals[k].get("SQ_WAVES", [0])))
for k in keys:
    if "ctn::" not in k:
        continue
    d = {c: sum(v) / len(v) for c, v in vals[k].items()}
    print(short(k))
    print("   " + "  ".join(f"{c}={d[c]:.4g}" for c in sorted(d)))
