"""Tabulate tools/gpu_variants.sh output: kernel avg us per variant (columns)."""
import re
import sys

txt = open(sys.argv[1]).read()
names, data = [], {}
for b in re.split(r"^== ", txt, flags=re.M)[1:]:
    lines = b.strip().split("\n")
    col = lines[0].split()[0]
    while col in data:
        col += "'"
    thr = re.search(r'ue": ([\d.]+)', lines[0])
    names.append(col)
    data[col] = {"utt/s": thr.group(1) if thr else "?"}
    for l in lines[1:]:
        m = re.search(r"([\d.]+) us avg.*?(?:void )?ctn::([^(]+)\(", l)
        if m:
            data[col][m.group(2).replace("unsigned short", "u16")] = m.group(1)
ks = ["utt/s"] + sorted({k for d in data.values() for k in d if k != "utt/s"})
w = max(len(k) for k in ks) + 1
print(" " * w + "".join(f"{n:>9}" for n in names))
for k in ks:
    print(f"{k:{w}}" + "".join(f"{data[n].get(k, '-'):>9}" for n in names))
