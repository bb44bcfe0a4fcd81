"""Instruction mix of a kernel's longest loop (the iteration of an iterative solver) in a code object.
usage: python tools/loop_mix.py <code object> <kernel-name substring>"""
import re
import subprocess
import sys
from collections import Counter


def rows_of(co, name):
    L = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                       text=True, check=True).stdout.split("\n")
    s = next(i for i, l in enumerate(L) if re.match(r"^[0-9a-f]+ <", l) and name in l)
    e = next((i for i in range(s + 1, len(L)) if re.match(r"^[0-9a-f]+ <", L[i])), len(L))
    rows = []
    for l in L[s + 1:e]:
        m = re.match(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):[^<]*(?:<[^+]*\+0x([0-9a-f]+)>)?", l)
        if m:
            rows.append((int(m.group(3), 16), m.group(1), m.group(2), m.group(4)))
    return rows


def main(co, name):
    rows = rows_of(co, name)
    base = rows[0][0]
    idx = {a - base: i for i, (a, _, _, _) in enumerate(rows)}
    best = None
    for i, (a, op, args, t) in enumerate(rows):
        if t and (op.startswith("s_cbranch") or op == "s_branch"):
            j = idx.get(int(t, 16))
            if j is not None and j < i and (best is None or i - j > best[1] - best[0]):
                best = (j, i)
    j, i = best
    seg = rows[j:i + 1]
    c = Counter(x[1] for x in seg)
    fma = sum(v for k, v in c.items() if "fma" in k or "fmac" in k or "fmamk" in k or "fmaak" in k)
    nops = sum(int(x[2].split()[0], 0) + 1 for x in seg if x[1] == "s_nop")
    print(f"{name}: kernel {len(rows)} instructions, main loop {len(seg)} (fma {fma}, dpp "
          f"{sum(1 for x in seg if '_dpp' in x[1])}, s_nop wait states {nops}, ds {sum(1 for x in seg if x[1].startswith('ds_'))})")
    print("  " + " ".join(f"{k}:{v}" for k, v in c.most_common(30)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
