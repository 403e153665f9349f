#!/usr/bin/env python3
"""Per-kernel register / spill / LDS figures of a built HIP object or library.

    python3 scripts/kernel_resources.py hb_mcmc_amd/lib/hb_kernels.o [name-regex]

Extracts the gfx950 code object from the object's .hip_fatbin section
(clang-offload-bundler) and prints, from the code-object metadata notes, every
kernel's VGPR / AGPR / SGPR counts, VGPR and SGPR spills, static LDS and
private segment size.  Kernel names are demangled.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_object(path: str, tmp: str) -> str:
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path, os.path.join(tmp, "junk")],
                   check=True, capture_output=True)
    co = os.path.join(tmp, "co.o")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                   check=True, capture_output=True)
    return co


def kernels(co: str):
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    cur = None
    for line in notes.splitlines():
        s = line.strip()
        if s.startswith("- .agpr_count:") or s.startswith(".agpr_count:"):
            if cur:
                yield cur
            cur = {}
        m = re.match(r"-?\s*\.(\w+):\s+(.*)$", s)
        if m and cur is not None:
            cur.setdefault(m.group(1), m.group(2))
    if cur:
        yield cur


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout
    return out.splitlines()


def main() -> None:
    path = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    with tempfile.TemporaryDirectory() as tmp:
        ks = [k for k in kernels(code_object(path, tmp)) if "name" in k]
    names = demangle([k["name"] for k in ks])
    rows = []
    for k, dn in zip(ks, names):
        if pat and not pat.search(dn):
            continue
        rows.append((dn, k.get("vgpr_count"), k.get("agpr_count"), k.get("sgpr_count"), k.get("vgpr_spill_count"),
                     k.get("sgpr_spill_count"), k.get("group_segment_fixed_size"), k.get("private_segment_fixed_size")))
    print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'vspl':>5} {'sspl':>5} {'lds':>6} {'priv':>5}  kernel")
    for dn, v, a, s, vs, ss, lds, pr in sorted(rows):
        dn = re.sub(r"\(.*\)$", "", dn)
        print(f"{v:>5} {a:>5} {s:>5} {vs:>5} {ss:>5} {lds:>6} {pr:>5}  {dn}")


if __name__ == "__main__":
    main()
