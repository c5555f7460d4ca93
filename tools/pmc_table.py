"""Per-kernel HBM traffic per launch (FETCH_SIZE x2 + WRITE_SIZE, gfx950) from rocprofv3 --pmc passes -> CSV."""
import csv, glob, os, sys
from collections import defaultdict
root, out = sys.argv[1], sys.argv[2]
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(out, "w", newline="") as fh:
    w = csv.writer(fh)
    w.writerow(["kernel", "launches", "fetch_bytes_per_launch_x2", "write_bytes_per_launch", "total_bytes_per_launch"])
    for k, d in sorted(vals.items(), key=lambda kv: -sum(kv[1].get("FETCH_SIZE", [0]))):
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        fe = 2 * 1024 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
        wr = 1024 * sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
        w.writerow([k[:120], len(d["FETCH_SIZE"]), round(fe), round(wr), round(fe + wr)])
