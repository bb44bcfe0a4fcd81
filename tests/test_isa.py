"""no product kernel contains a flat memory instruction -- in particular no flat access into a
lane's private segment (the hazard profiles/r04_ikc_fault.txt named: the out-of-line trig call wrote its
results through flat pointers to the caller's stack).  tools/isa_check.py disassembles the gfx950 code objects
of the engine's kernel translation units (the generic kernels; the plan-specialised ones are checked on a GPU
box from their dumped code objects, profiles/r05_isa_check.txt).  CPU only: needs the in-tree build."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "kinematics.jl_amd", "lib", "obj")


@pytest.mark.skipif(not os.path.exists(os.path.join(OBJ, "kinhip_ik.o")), reason="needs the in-tree build objects")
def test_no_flat_instruction_in_generic_kernels():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_check.py")], capture_output=True, text=True,
                       timeout=600)
    print(r.stdout[-2000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "kinhip_ikt.o" in r.stdout and "kinhip_ik.o" in r.stdout
