"""The one A/B driver: runs a workload script once per setting of the A/B knobs, against
the tools-only library lib/libkinhip_ab.so (`make -C kinematics.jl_amd/csrc ab`, -DKINHIP_AB_KNOBS=1).
The product library libkinhip.so never reads these variables (kinhip_internal.h ab_env).

    python tools/ab.py <workload> [--reps R] [SETTING ...]
      workload: ik (tools/ik_ab.py: config-4 IK), coll (tools/coll_spec_ab.py: config-5 k_coll legs),
                fk (tools/fk_legs_ab.py: headline FK + J and config 2), jl (tools/jl_layout_ab.py: FK + J at
                ld = N, the Julia shim's layout), scene (tools/scene_ab.py: the f2 door sweep), cik (tools/cik_ab.py:
                the f2 / f3 legs, stage-2 times)
      SETTING:  "NAME=VALUE[,NAME=VALUE...]" -- one run per setting; "base" = no knob
    e.g. python tools/ab.py ik base KINHIP_IK_TWO_PHASE=0 KINHIP_IK_GROUP=2,KINHIP_IK_TWO_PHASE=0
         python tools/ab.py coll base "KINHIP_JIT_DEFS=-DKINHIP_AABB_UNROLL=1" KINHIP_COLL_FAST_TRIG=0

Knobs (all read only by the A/B build): KINHIP_IK_GROUP, KINHIP_IK_RESIDENT, KINHIP_IK_QUEUE,
KINHIP_IK_TWO_PHASE, KINHIP_IK_TP_QUEUE (IK schedule), KINHIP_IKC_GROUP (collision-aware IK lanes), KINHIP_FK_PER_LANE (FK grid), KINHIP_JIT_IK_WAVES,
KINHIP_JIT_COLL_WAVES (occupancy), KINHIP_COLL_FAST_TRIG, KINHIP_IK_FAST_ATAN (arithmetic variants), KINHIP_SCENE_LDS (scene frames in LDS),
KINHIP_JIT_SLP, KINHIP_JIT_DEFS, KINHIP_JIT_OPTS (compiler options / definitions), KINHIP_JIT_DUMP
(keep the generated source).  Every run prints its workload's own result line prefixed by the setting."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = {"ik": "ik_ab.py", "coll": "coll_spec_ab.py", "fk": "fk_legs_ab.py", "jl": "jl_layout_ab.py",
           "scene": "scene_ab.py", "cik": "cik_ab.py"}


def main(argv):
    if len(argv) < 2 or argv[1] not in SCRIPTS:
        print(__doc__)
        return 2
    args = argv[2:]
    reps = 1
    if args[:1] == ["--reps"]:
        reps, args = int(args[1]), args[2:]
    lib = os.path.join(ROOT, "kinematics.jl_amd", "lib", "libkinhip_ab.so")
    if not os.path.exists(lib):
        print(f"{lib} is missing: make -C kinematics.jl_amd/csrc ab")
        return 2
    script = os.path.join(ROOT, "tools", SCRIPTS[argv[1]])
    rc = 0
    for rep in range(reps):
        for setting in args or ["base"]:
            env = dict(os.environ, KINHIP_LIB=lib, AB_SPEC=os.environ.get("AB_SPEC", "1"))
            if setting != "base":
                for kv in setting.split(","):
                    k, v = kv.split("=", 1)
                    env[k] = v
            r = subprocess.run([sys.executable, "-u", script], env=env, capture_output=True, text=True, timeout=600)
            lines = [l for l in r.stdout.splitlines() if l.strip()]
            print(f"[{setting}] rep {rep}: " + (lines[-1] if lines else f"(no output, rc {r.returncode})"), flush=True)
            if r.returncode != 0:
                print(r.stderr[-2000:])
                rc = r.returncode
                break
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv))
