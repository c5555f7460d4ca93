"""Instruction mix of the loops of one kernel in a hipcc -S listing.

usage: python tools/isa_loops.py <file.s> <kernel-symbol-substring>
For every loop (a label followed later by a branch back to it) that contains an
MFMA, prints the instruction-class counts of the loop body.
"""
import re
import sys
from collections import Counter

path, sub = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sub in l and l.rstrip().endswith(":") or (sub in l and re.match(r"^_Z\S+:", l)))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
labels = {}
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):", l)
    if m:
        labels[m.group(1)] = i
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", l)
    if not m:
        continue
    tgt = m.group(1) or m.group(2)
    j = labels.get(tgt)
    if j is None or j >= i:
        continue
    region = body[j:i + 1]
    ops = [r.split()[0] for r in region if r.startswith("\t") and r.split() and not r.split()[0].startswith(";")]
    if not any(o.startswith("v_mfma") for o in ops):
        continue
    c = Counter(ops)
    cls = Counter()
    for o, n in c.items():
        k = ("mfma" if o.startswith("v_mfma") else "valu" if o.startswith("v_") else "salu" if o.startswith("s_") and not o.startswith("s_waitcnt") else
             "wait" if o.startswith("s_waitcnt") else "lds" if o.startswith("ds_") else "vmem" if o.startswith(("global_", "buffer_")) else "other")
        cls[k] += n
    print(f"loop {tgt} lines {j}-{i}: " + " ".join(f"{k}={v}" for k, v in sorted(cls.items())))
    print("   top valu: " + " ".join(f"{o}:{n}" for o, n in c.most_common(40) if o.startswith("v_") and not o.startswith("v_mfma"))[:600])
