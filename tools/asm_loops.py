#!/usr/bin/env python3
"""Instruction mix of the hottest loops of a kernel in a hipcc -S listing.
usage: asm_loops.py file.s kernel_substring [--top 3]"""
import re
import sys
from collections import Counter

path, pat = sys.argv[1], sys.argv[2]
top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 3
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.size") or lines[i].startswith(".Lfunc_end"))
body = lines[start:end]
# blocks
blocks, cur, name = [], [], "entry"
for l in body:
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        blocks.append((name, cur)); name, cur = m.group(1), []
    else:
        cur.append(l.strip())
blocks.append((name, cur))

def cat(ins):
    op = ins.split()[0] if ins and not ins.startswith(";") and not ins.startswith(".") else ""
    if not op: return None
    if op.startswith("v_mfma"): return "mfma"
    if op.startswith("ds_read") or op.startswith("ds_load"): return "ds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"): return "ds_write"
    if op.startswith("global_load") or op.startswith("buffer_load"): return "vmem_load"
    if op.startswith("global_store") or op.startswith("buffer_store") or op.startswith("global_atomic"): return "vmem_store"
    if op.startswith("v_"): return "valu"
    if op.startswith("s_waitcnt"): return "waitcnt"
    if op.startswith("s_barrier"): return "barrier"
    if op.startswith("s_"): return "salu"
    return "other"

stats = []
for n, b in blocks:
    c = Counter(x for x in map(cat, b) if x)
    ops = Counter(i.split()[0] for i in b if i and cat(i) == "valu")
    stats.append((c.get("mfma", 0), n, c, ops))
stats.sort(key=lambda s: -s[0])
for m, n, c, ops in stats[:top]:
    print(n, dict(c))
    print("   valu:", ops.most_common(25))
