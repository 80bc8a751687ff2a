"""Instruction mix of a kernel's main tile loop, per s_barrier-delimited segment, from a hipcc
--save-temps .s file: python scripts/loop_mix.py <file.s> <kernel-symbol-substring>"""
import collections
import re
import sys

path, sub = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(sub) + r"\S*:", l))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
body = lines[start:end]
# the Depth=1 loop holding the most barriers
heads = [i for i, l in enumerate(body) if "Loop Header: Depth=1" in l]
best = None
for h in heads:
    label = body[h].split(":")[0].strip()
    back = max((i for i in range(h, len(body)) if re.search(r"s_c?branch\w* " + re.escape(label) + r"\b", body[i])),
               default=None)
    if back is None:
        continue
    nb = sum("s_barrier" in body[i] for i in range(h, back))
    if best is None or nb > best[2]:
        best = (h, back, nb)
h, back, nb = best
segs = [collections.Counter()]
for l in body[h:back + 1]:
    l = l.strip()
    if not l or l[0] in ";.":
        continue
    op = l.split()[0]
    if op == "s_barrier":
        segs.append(collections.Counter())
        continue
    c = segs[-1]
    if "mfma" in op:
        c["mfma"] += 1
    elif op.startswith("v_exp"):
        c["exp"] += 1
    elif op.startswith("v_"):
        c["valu"] += 1
        c["v:" + op] += 1
    elif op.startswith("ds_read"):
        c["ds_read"] += 1
    elif op.startswith("ds_write"):
        c["ds_write"] += 1
    elif op.startswith(("buffer_", "global_")):
        c["vmem"] += 1
    elif op.startswith("s_"):
        c["salu"] += 1
print(f"{sub}: loop of {back - h} lines, {nb} barriers (static counts, all branches included)")
for i, c in enumerate(segs):
    print(f" segment {i}:", {k: c[k] for k in ("mfma", "exp", "valu", "ds_read", "ds_write", "vmem", "salu")})
    print("    valu:", sorted([(v, k[2:]) for k, v in c.items() if k.startswith("v:")], reverse=True)[:10])
