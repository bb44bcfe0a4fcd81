"""Rebuild a dumped specialised source (KINHIP_JIT_DUMP) against the current device headers and
compile it offline with hiprtc (tools/jit_rtc_check.cpp) for ISA / register inspection.
usage: python tools/jit_offline.py <dump.hip> <out.hip>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
inc = open(os.path.join(ROOT, "kinematics.jl_amd", "lib", "obj", "kinhip_jit_src.inc")).read()
dev = inc[inc.index('R"KINHIPJIT(') + len('R"KINHIPJIT('):inc.rindex(')KINHIPJIT"')]
src = open(sys.argv[1]).read()
tail = src[src.index("namespace kinhip {\ntemplate <class X, int N> struct KArr"):]
open(sys.argv[2], "w").write(dev + tail)
