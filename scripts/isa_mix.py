"""Instruction mix of one kernel in a gfx950 .s file, per basic block.
usage: python scripts/isa_mix.py file.s kernel_symbol [top_blocks]"""
import re
import sys
from collections import Counter

path, sym = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 12
lines = open(path).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
blocks, cur, name = [], [], "entry"
for l in lines[start + 1:end + 1]:
    s = l.strip()
    if re.match(r"^\.?[A-Za-z0-9_$.]+:", s) and not s.startswith(";"):
        blocks.append((name, cur))
        name, cur = s.split(":")[0], []
        continue
    if not s or s.startswith(";") or s.startswith("."):
        continue
    cur.append(s.split()[0])
blocks.append((name, cur))


def cls(op):
    if op.startswith("v_") and "f64" in op:
        return "valu_f64"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


tot = Counter()
for n, ops in blocks:
    tot.update(cls(o) for o in ops)
print("kernel total:", dict(tot), "instrs", sum(tot.values()))
big = sorted(blocks, key=lambda b: -len(b[1]))[:top]
for n, ops in big:
    c = Counter(cls(o) for o in ops)
    f64 = Counter(o for o in ops if cls(o) == "valu_f64")
    print(f"{n:24s} {len(ops):5d}  {dict(c)}")
    print("     top f64:", f64.most_common(8))
