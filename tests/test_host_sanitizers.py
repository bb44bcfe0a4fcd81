"""The engine's host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

`make -C kinematics.jl_amd/csrc asan` builds tests/asan/kin_host_harness.cpp against the host translation
units of libkinhip (URDF reader, tree validation, rptable, add_link, plan / collision-plan staging, the
JIT source emitter), with the gfx950 launchers stubbed (tests/asan/launch_stubs.cpp).  The harness runs
the golden URDFs, seeded random trees (tests/randtree.py) and thousands of seeded corruptions of them
(truncations, XML-significant byte flips, deleted / duplicated spans, random bytes); any sanitizer
report or a status outside kin_status aborts it."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, golden
from randtree import random_urdf

CSRC = os.path.join(ROOT, "kinematics.jl_amd", "csrc")
HARNESS = os.path.join(ROOT, "kinematics.jl_amd", "lib", "asan", "kin_host_harness")


@pytest.fixture(scope="module")
def harness():
    subprocess.check_call(["make", "-s", "-C", CSRC, "asan"])
    return HARNESS


def _run(harness, files, mutants, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness, "--mutants", str(mutants), "--seed", str(seed), *files], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    return r.stdout


def test_golden_urdfs_and_corruptions(harness):
    out = _run(harness, [golden("fetch.urdf"), golden("fridge.urdf"), golden("pr2_torso_rarm.urdf")], 400, 1)
    assert "parsed" in out


def test_random_trees_and_corruptions(harness, tmp_path):
    rng = np.random.default_rng(2026)
    files = []
    for k in range(12):
        p = tmp_path / f"t{k}.urdf"
        p.write_text(random_urdf(rng, int(rng.integers(2, 40)), chain_bias=float(rng.uniform(0.3, 0.95))))
        files.append(str(p))
    malformed = ["<robot><link", "<robot name='x'><link name='a'/><joint name='j' type='floating'><parent link='a'/>"
                 "<child link='b'/></joint></robot>", "<?xml version='1.0'?><!-- c --><robot name='r'><link name='a'/>"
                 "</robot>", "<robot><link name='a'/><link name='a'/></robot>", "<robot><joint name='j' type='fixed'>"
                 "<parent link='zz'/><child link='yy'/></joint></robot>", "<![CDATA[<robot>]]>", "&amp;&lt;&#x41;",
                 "<robot><link name='a'><collision><geometry><box size='1 2'/></geometry></collision></link></robot>"]
    for k, t in enumerate(malformed):
        p = tmp_path / f"m{k}.urdf"
        p.write_text(t)
        files.append(str(p))
    _run(harness, files, 60, 7)
