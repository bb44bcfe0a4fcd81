"""Instruction histogram / loop listing for one kernel in the `make asm` output.
usage: python tools/asm_kernel.py <substring of mangled name> [--loops]"""
import re
import sys
from collections import Counter

import glob
pat = sys.argv[1]
lines = []
for S in sorted(glob.glob("kinematics.jl_amd/lib/obj/kinhip_*.s")):
    lines += open(S).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and pat in l)
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
body = [l.split(";")[0].strip() for l in lines[start:end]]
ins = [l for l in body if l and not l.startswith(".") and not l.endswith(":")]
print(lines[start][:120], "instructions:", len(ins))
c = Counter(l.split()[0] for l in ins)
print(" ".join(f"{k}:{v}" for k, v in c.most_common(40)))
if "--loops" in sys.argv:
    labels = {l[:-1]: i for i, l in enumerate(body) if l.endswith(":")}
    for i, l in enumerate(body):
        m = re.match(r"s_cbranch_\w+\s+(\S+)", l) or re.match(r"s_branch\s+(\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            blk = [x for x in body[labels[m.group(1)]:i + 1] if x and not x.startswith(".") and not x.endswith(":")]
            cc = Counter(x.split()[0] for x in blk)
            print(f"loop {m.group(1)}: {len(blk)} instr;", " ".join(f"{k}:{v}" for k, v in cc.most_common(25)))
