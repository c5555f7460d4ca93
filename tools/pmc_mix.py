"""Per-kernel issue/wait mix from rocprofv3 --pmc passes (tools/gpu_pmc_model.sh).

For each ctn kernel: mean per dispatch of the SQ counters, and the fractions of
wave cycles spent issuing (ACTIVE_INST_ANY), stalled on dependencies/pipes
(WAIT_INST_ANY) and parked on waitcnt/barriers (WAIT_ANY), plus instruction
counts per wave.
"""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, d in vals.items():
    if "ctn::" not in k:
        continue
    m = {c: sum(v) / len(v) for c, v in d.items()}
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    waves = m.get("SQ_WAVES", 0) or 1
    rows.append((m.get("SQ_WAVE_CYCLES", 0), k, m, wc, waves))
rows.sort(reverse=True)
for _, k, m, wc, waves in rows[:14]:
    name = k.replace("ctn::", "").replace("unsigned short", "bf16")[:64]
    print(f"{name}")
    print(f"   issue {m.get('SQ_ACTIVE_INST_ANY',0)/wc:5.2f}  dep/pipe-stall {m.get('SQ_WAIT_INST_ANY',0)/wc:5.2f}  "
          f"parked {m.get('SQ_WAIT_ANY',0)/wc:5.2f} | per wave: valu {m.get('SQ_INSTS_VALU',0)/waves:7.0f} "
          f"mfma {m.get('SQ_INSTS_MFMA',0)/waves:6.0f} lds {m.get('SQ_INSTS_LDS',0)/waves:6.0f} salu {m.get('SQ_INSTS_SALU',0)/waves:6.0f} "
          f"vmem {m.get('SQ_INSTS_VMEM',0)/waves:6.0f} | lds-conflict/idx {m.get('SQ_LDS_BANK_CONFLICT',0)/(m.get('SQ_LDS_IDX_ACTIVE',0) or 1):.3f} "
          f"waves {waves:.0f} wavecyc/wave {wc/waves:.0f}")
