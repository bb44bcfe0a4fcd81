"""Rebuild a dumped specialised source (KINHIP_JIT_DUMP) against the CURRENT device headers (csrc/, as the
Makefile embeds them) and compile it offline with hiprtc (tools/jit_rtc_check.cpp) for ISA / register
inspection -- no GPU needed.
usage: python tools/jit_offline.py <dump.hip> <out.co> [kernel-name-substring ...] [--set 'p.nzrow[0] = 1u;' ...]
  kernel-name substrings: keep only those extern "C" kernels (all if none)."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.environ.get("KINHIP_CSRC", os.path.join(ROOT, "kinematics.jl_amd", "csrc"))  # (another tree: A/B)
HDRS = ["kinhip_prog.h", "kinhip_device.h", "kinhip_fk_dev.h", "kinhip_ik_dev.h", "kinhip_coll_dev.h", "kinhip_ikt_dev.h"]
OPTS = ["-ffp-contract=fast-honor-pragmas", "-DKINHIP_COLL_SOFF=1", "-DKINHIP_COLL_FAST_TRIG=1",
        "-DKINHIP_IK_FAST_ATAN=1"]


def device_source():
    out = []
    for h in HDRS:
        for line in open(os.path.join(CSRC, h)):
            if line.startswith("#pragma once") or line.startswith('#include "kinhip_'):
                continue
            out.append(line)
    return "".join(out)


def main(argv):
    args, sets, keep = argv[3:], [], []
    i = 0
    while i < len(args):
        if args[i] == "--set":
            sets.append(args[i + 1])
            i += 2
        else:
            keep.append(args[i])
            i += 1
    src = open(argv[1]).read()
    tail = src[src.index("namespace kinhip {\ntemplate <class X, int N> struct KArr"):]
    if sets:  # extra table assignments (e.g. fields a newer KIkcProg has and the dump predates)
        k = tail.index("constexpr KIkcProg")  # (the collision-aware IK program: kIP)
        j = tail.index("  return p;\n}();", k)
        tail = tail[:j] + "".join("  " + s + "\n" for s in sets) + tail[j:]
    if keep:
        parts = re.split(r'(?=extern "C" __global__)', tail)
        name = lambda p: p.split(" void ", 1)[1].split("(")[0]
        tail = parts[0] + "".join(p for p in parts[1:] if any(k in name(p) for k in keep))
    path = argv[2] + ".hip"
    open(path, "w").write(device_source() + tail)
    tool = "/tmp/jit_rtc_check"
    if not os.path.exists(tool):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O2", os.path.join(ROOT, "tools", "jit_rtc_check.cpp"), "-o", tool,
                        "-lhiprtc"], check=True)
    extra = os.environ.get("KINHIP_OFFLINE_DEFS", "").split()  # (e.g. -DKINHIP_IKT_SECT=5)
    r = subprocess.run([tool, path, argv[2]] + OPTS + extra, capture_output=True, text=True)
    sys.stderr.write(r.stderr[-4000:])
    return r.returncode


if __name__ == "__main__":
    sys.exit(main(sys.argv))
