"""Per-kernel MFMA utilisation and issue breakdown from tools/gpu_pmc_mfma.sh passes.

mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs): the
fraction of all SIMD-cycles of the dispatch in which a matrix core was busy
(GRBM_GUI_ACTIVE sums the 8 XCDs; MI355X_MICROARCH.md §DVFS, §rocprofv3 PMC).
Wave-cycle buckets (quad-cycles): WAIT_ANY (parked on s_waitcnt / barrier),
WAIT_INST_ANY (issue stall), ACTIVE_INST_ANY (issuing)."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
json_out = sys.argv[2] if len(sys.argv) > 2 else None
KINDS = {   # bench.py timer kinds (include/ctn.h CTN_TIMER_*) -> kernel name (bf16, gLN c2 shape)
    "1": "gemm_ws_kernel<0, 0, 1, 2, 8, 16, 2, 1>",
    "2": "dw_fwd_wave_kernel<0, false>",
    "3": "gemm_dual_ws_kernel<0, ",   # the wave-specialised pair-A dual (gLN)
    "4": "dw_bwd_wave_kernel<0, false>",
    "5": "gemm_ws_kernel<3, 0, 2, 2, 16, 8, 1, 1>",
    "6": "gemm_cols_kernel<unsigned short, 0, 0, 0>",
    "7": "gemm_ws_kernel<2, 0, 2, 2, 16, 8, 1, 1>",
}
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "ctn::" not in k:
            continue
        k = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ctn::", "").replace("ctn::", "")
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
def m(d, c):
    v = d.get(c)
    return sum(v) / len(v) if v else float("nan")
print("%-46s %6s %9s %7s %7s %7s %7s %7s %7s" % ("kernel", "n", "mfma/lch", "util%", "wait%", "stall%", "issue%", "valu/mf", "lds/mf"))
rows = []
for k, d in vals.items():
    n = len(d.get("SQ_INSTS_MFMA", [0]))
    cyc = m(d, "GRBM_GUI_ACTIVE") / 8.0
    util = m(d, "SQ_VALU_MFMA_BUSY_CYCLES") / (cyc * 1024) * 100 if cyc == cyc and cyc > 0 else float("nan")
    wc = m(d, "SQ_WAVE_CYCLES")
    mf = m(d, "SQ_INSTS_MFMA")
    rows.append((cyc, "%-46s %6d %9.0f %7.1f %7.1f %7.1f %7.1f %7.2f %7.2f" % (
        k[:46], n, mf, util, 100 * m(d, "SQ_WAIT_ANY") / wc, 100 * m(d, "SQ_WAIT_INST_ANY") / wc,
        100 * m(d, "SQ_ACTIVE_INST_ANY") / wc, m(d, "SQ_INSTS_VALU") / mf if mf else float("nan"),
        m(d, "SQ_INSTS_LDS") / mf if mf else float("nan"))))
for _, r in sorted(rows, reverse=True):
    print(r)
if json_out:
    import json
    out = {}
    for kind, pat in KINDS.items():
        for k, d in vals.items():
            if k.startswith(pat) or k == pat:
                cyc = m(d, "GRBM_GUI_ACTIVE") / 8.0
                busy = m(d, "SQ_VALU_MFMA_BUSY_CYCLES")
                out[kind] = {"kernel": k, "mfma_util": round(busy / (cyc * 1024), 4), "mfma_per_launch": m(d, "SQ_INSTS_MFMA"),
                             "mfma_busy_cycles": busy, "gui_active_per_xcd": cyc,
                             "note": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 XCDs * 1024 SIMDs), per launch"}
    json.dump(out, open(json_out, "w"), indent=1)
