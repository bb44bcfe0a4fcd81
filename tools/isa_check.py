"""ISA check of every product kernel: no flat memory instruction -- in particular no flat
access into a lane's private segment, the round-4 fault's named hazard (profiles/r04_ikc_fault.txt) -- and
the out-of-line calls (s_swappc) listed per kernel.  Disassembles the gfx950 code objects of the library's
object files (the generic kernels) and any code objects given on the command line (the hiprtc-specialised
kernels, dumped on a GPU box by the A/B build with KINHIP_JIT_CODE_DUMP=<prefix>).

    python tools/isa_check.py [more.co ...]      (exit status 1 if any flat instruction is found)"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects_of(obj, tmp):
    """The gfx950 device code object inside a host object file (its .hip_fatbin offload bundle)."""
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", obj, os.path.join(tmp, "x.o")],
                   check=True, capture_output=True)
    co = os.path.join(tmp, os.path.basename(obj) + ".gfx950.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}", f"--output={co}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True, capture_output=True)
    return co


def scan(co):
    """-> {function: (instructions, flat instructions, s_swappc count)}"""
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True, capture_output=True,
                         text=True).stdout
    funcs, cur = {}, None
    for line in out.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            funcs[cur] = [0, 0, 0]
            continue
        if cur is None or not line.startswith("\t"):
            continue
        ins = line.strip().split()[0] if line.strip() else ""
        if not ins or ins.startswith("//"):
            continue
        f = funcs[cur]
        f[0] += 1
        if ins.startswith("flat_"):
            f[1] += 1
        if ins.startswith("s_swappc"):
            f[2] += 1
    return funcs


def main(argv):
    obj_dir = os.path.join(ROOT, "kinematics.jl_amd", "lib", "obj")
    objs = [os.path.join(obj_dir, f"kinhip_{k}.o") for k in ("fk", "ik", "ikt", "coll")]  # (the product's)
    objs = [o for o in objs if os.path.exists(o)]  # (lib/obj stays in the build container: not on a GPU box)
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        sources = [(os.path.basename(o), code_objects_of(o, tmp)) for o in objs] + [(os.path.basename(c), c)
                                                                                  for c in argv[1:]]
        for name, co in sources:
            funcs = scan(co)
            kernels = {k: v for k, v in funcs.items() if not k.endswith((".kd",))}
            n_flat = sum(v[1] for v in kernels.values())
            calls = sum(v[2] for v in kernels.values())
            callers = sum(1 for v in kernels.values() if v[2])
            print(f"{name}: {len(kernels)} functions, {sum(v[0] for v in kernels.values())} instructions, "
                  f"flat {n_flat}, s_swappc {calls} in {callers} functions")
            for k, v in kernels.items():
                if v[1]:
                    print(f"  FLAT {v[1]:5d}  {k[:150]}")
            bad += n_flat
    print("flat instructions in product kernels:", bad, "(must be 0)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
