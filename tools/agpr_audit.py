"""Audit a kernel that owns accumulator registers by name (prefill_x64_kernel): every v_accvgpr_* and every AGPR
operand outside the kernel's own inline-asm statements would be hipcc's, i.e. a collision.  Also reports spills.
Usage: python3 tools/agpr_audit.py file.s kernel_substring"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r"^(_Z\w*" + sys.argv[2] + r"\w*):", s, re.M)
body = s[m.end(): s.find(".Lfunc_end", m.end())]
inside = False
bad = []
for ln in body.splitlines():
    t = ln.strip()
    if t.startswith(";;#ASMSTART"):
        inside = True
        continue
    if t.startswith(";;#ASMEND"):
        inside = False
        continue
    if not t or t.startswith((";", ".")) or inside:
        continue
    if "accvgpr" in t or re.search(r"\ba\[?\d", t):
        bad.append(t)
print(f"compiler-generated AGPR instructions: {len(bad)}")
for t in bad[:20]:
    print("  ", t)
print("scratch:", len(re.findall(r"scratch_", body)))
sys.exit(1 if bad else 0)
