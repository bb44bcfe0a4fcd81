"""The C-ABI driven from plain C (examples/kin_c_demo.c, built by __graft_entry__.build() with gcc):
fetch.urdf through the native loader, a specialised FK + Jacobian plan, device results checked
against the reference's q = 0 gripper pose -- the path a Julia ccall / cgo / JNI binding takes."""
import os
import subprocess

import pytest

from conftest import ROOT, golden

DEMO = os.path.join(ROOT, "kinematics.jl_amd", "lib", "kin_c_demo")


def test_c_demo_built():
    assert os.path.exists(DEMO), "run __graft_entry__.build() (make -C kinematics.jl_amd/csrc)"


@pytest.mark.gpu
def test_c_demo_runs_on_device():
    r = subprocess.run([DEMO, golden("fetch.urdf")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK" in r.stdout
