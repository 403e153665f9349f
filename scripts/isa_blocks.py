"""Basic blocks of one kernel in a gfx950 .s file, in layout order, split at
branches: (label, instructions, fp64 instructions, branch).
usage: python scripts/isa_blocks.py file.s kernel_symbol_prefix [max_rows]"""
import re
import sys

path, pref = sys.argv[1], sys.argv[2]
rows = int(sys.argv[3]) if len(sys.argv) > 3 else 80
lines = open(path).read().splitlines()
sym = [l for l in lines if l.startswith(pref) and l.rstrip().endswith(":") or (l.startswith(pref) and ": ;" in l)][0].split(":")[0]
s = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
e = next(i for i in range(s, len(lines)) if "s_endpgm" in lines[i] or lines[i].startswith(".Lfunc_end"))
name, cnt, f64, out = "entry", 0, 0, []
for l in lines[s + 1:e + 1]:
    t = l.strip()
    if re.match(r"^\.LBB[0-9_]+:", t):
        out.append((name, cnt, f64, ""))
        name, cnt, f64 = t.split(":")[0], 0, 0
        continue
    if not t or t.startswith(";") or t.startswith("."):
        continue
    cnt += 1
    f64 += "f64" in t.split()[0]
    if t.startswith("s_cbranch") or t.startswith("s_branch") or t.startswith("s_swappc") or t.startswith("s_setpc"):
        out.append((name, cnt, f64, t))
        name, cnt, f64 = name + "+", 0, 0
out.append((name, cnt, f64, ""))
for o in out[:rows]:
    print("%-16s %5d %5d  %s" % o)
