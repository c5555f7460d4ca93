"""HBM bytes of one whole training step from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes, against the step's algorithmic bytes (SURVEY.md §8d model).

usage: python tools/pmc_step.py <pmc dir with p*/run_counter_collection.csv>
                                <kernel_trace.csv of a --kernel-trace run of the same config>
                                [algorithmic GB per step] [out.json]

Per kernel name: mean FETCH_SIZE (x2, the gfx950 wide-read correction of
MI355X_MICROARCH.md §HBM/rocprofv3) + WRITE_SIZE per dispatch, KiB -> B.  Launches
per step: the dispatches between the last two Adam launches of the trace (one
steady-state step).  Kernels that read with narrower than 16-byte lanes are
over-corrected by the x2; every hot kernel here reads 16 B per lane.
"""
import csv
import glob
import json
import os
import sys
from collections import Counter, defaultdict


def main():
    pmc_dir, trace = sys.argv[1], sys.argv[2]
    alg_gb = float(sys.argv[3]) if len(sys.argv) > 3 else None
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if "adam" in r["Kernel_Name"]]
    if len(adam) < 2:
        sys.exit("need two Adam launches in the trace")
    step = Counter(r["Kernel_Name"] for r in rows[adam[-2] + 1:adam[-1] + 1])
    per, total, missing = {}, 0.0, []
    for name, n in step.items():
        d = vals.get(name)
        if not d or "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            missing.append(name)
            continue
        b = (2.0 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) + sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])) * 1024
        per[name] = {"launches_per_step": n, "bytes_per_launch": b, "bytes_per_step": b * n}
        total += b * n
    out = {"step_bytes": total, "step_GB": total / 1e9, "algorithmic_GB": alg_gb,
           "ratio": (total / 1e9 / alg_gb) if alg_gb else None, "kernels_without_counters": missing,
           "kernels": dict(sorted(per.items(), key=lambda kv: -kv[1]["bytes_per_step"]))}
    print(f"step HBM traffic {total / 1e9:.2f} GB" + (f" vs {alg_gb:.2f} GB algorithmic ({total / 1e9 / alg_gb:.3f}x)"
                                                       if alg_gb else ""))
    for name, v in list(out["kernels"].items())[:10]:
        print(f"  {v['bytes_per_step'] / 1e9:7.2f} GB  {v['launches_per_step']:4d} x {v['bytes_per_launch'] / 1e6:8.1f} MB  "
              f"{name[:90]}")
    if len(sys.argv) > 4:
        with open(sys.argv[4], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
