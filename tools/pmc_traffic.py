"""HBM traffic per launch of the bench.py timer kernels from rocprofv3 --pmc passes.

usage: python tools/pmc_traffic.py <dir with p*/run_counter_collection.csv> [out.json]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Per MI355X_MICROARCH.md
(HBM / rocprofv3): on gfx950 FETCH_SIZE reports exactly half the bytes of a
wide (16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is
exact for 16 B/lane streaming stores.  Every timed kernel reads and writes
with 16 B/lane accesses.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KINDS = {   # bench.py timer kinds (include/ctn.h CTN_TIMER_*) -> kernel name (bf16, gLN c2 shape)
    "1": "ctn::gemm_ws_kernel<0, 0, 1, 2, 8, 16, 2, 1>",
    "2": "dw_fwd_wave_kernel<0, false>",
    "3": "gemm_dual_ws_kernel<0, ",   # the wave-specialised pair-A dual (gLN)
    "4": "dw_bwd_wave_kernel<0, false>",
    "5": "ctn::gemm_ws_kernel<3, 0, 2, 2, 16, 8, 1, 1>",
    "6": "ctn::gemm_cols_kernel<unsigned short, 0, 0, 0>",
    "7": "ctn::gemm_ws_kernel<2, 0, 2, 2, 16, 8, 1, 1>",
}


def main():
    root = sys.argv[1]
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for kind, pat in KINDS.items():
        names = [n for n in vals if pat in n]
        if not names:
            continue
        d = vals[names[0]]
        if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
            continue
        fetch = 2.0 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024
        write = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024
        out[kind] = {"bytes": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
                     "kernel": pat, "launches": len(d["FETCH_SIZE"]),
                     "note": "per launch; FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->B"}
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(js + "\n")


if __name__ == "__main__":
    main()
