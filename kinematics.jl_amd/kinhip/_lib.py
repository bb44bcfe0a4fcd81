"""ctypes binding of libkinhip.so (the C-ABI declared in include/kinhip.h).

The library is built in-tree (``kinematics.jl_amd/lib/libkinhip.so``) by
``__graft_entry__.build()``.  There is no fallback: if it is missing, loading
fails loudly.  ``torch`` is imported first so that the library binds to the
HIP runtime torch already loaded (same soname), which lets torch device
pointers and streams cross the boundary.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the HIP library: shared runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KINHIP_LIB") or os.path.normpath(os.path.join(_HERE, "..", "lib", "libkinhip.so"))

KIN_OK = 0
KIN_E_INVALID, KIN_E_KEY, KIN_E_METHOD, KIN_E_DEVICE = -1, -2, -3, -4
KIN_E_UNSUPPORTED, KIN_E_NOMEM, KIN_E_PARSE, KIN_E_IO = -5, -6, -7, -8
KIN_F32, KIN_F64 = 0, 1
KIN_JOINT_FIXED, KIN_JOINT_REVOLUTE, KIN_JOINT_PRISMATIC = 0, 1, 2
KIN_WITH_ROT, KIN_RPY_JAC, KIN_ZERO_FILL = 1, 2, 4
KIN_SPEC_FK, KIN_SPEC_IK, KIN_SPEC_NAKAMURA, KIN_SPEC_COLL, KIN_SPEC_IK_COLL = 1, 2, 4, 8, 16
KIN_SPEC_IK_COLL_SCENE = 32
ABI_VERSION = 2  # KINHIP_ABI_VERSION of include/kinhip.h (kin_ik_params layout)

# every entry point include/kinhip.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "kin_abi_version", "kin_last_error", "kin_limits",
    "kin_model_create", "kin_model_destroy", "kin_model_num_links", "kin_model_num_joints",
    "kin_model_set_angles", "kin_model_is_relevant", "kin_model_add_link",
    "kin_urdf_parse_file", "kin_urdf_parse_string", "kin_urdf_destroy", "kin_urdf_tree",
    "kin_urdf_link_name", "kin_urdf_joint_name", "kin_urdf_find_link", "kin_urdf_find_joint",
    "kin_urdf_link_box",
    "kin_plan_create", "kin_plan_destroy", "kin_plan_shape", "kin_plan_run", "kin_plan_run_tiled",
    "kin_plan_specialize", "kin_plan_specialized", "kin_jit_selfcheck",
    "kin_get_transform_batch", "kin_get_jacobian_batch",
    "kin_ik_dls_batch", "kin_ik_dls_batch_from", "kin_ik_dls_batch_trace", "kin_point_ik_nakamura_batch",
    "kin_sdf_create_boxes", "kin_sdf_destroy", "kin_coll_plan_create", "kin_coll_batch",
    "kin_ineq_const_batch", "kin_pose_const_batch",
    "kin_coll_ik_plan_create", "kin_ik_coll_batch", "kin_ik_coll_batch_scene", "kin_sdf_create_attached",
    "kin_coll_batch_scene", "kin_plan_ik_sched_stats", "kin_plan_specialize_scene", "kin_ik_coll_batch_alt",
]


class KinError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"kinhip error {code}: {msg}")
        self.code = code


class TreeDesc(C.Structure):
    _fields_ = [("n_links", C.c_int32), ("n_joints", C.c_int32),
                ("joint_type", C.c_void_p), ("joint_plink", C.c_void_p), ("joint_clink", C.c_void_p),
                ("joint_pose", C.c_void_p), ("joint_axis", C.c_void_p),
                ("joint_lower", C.c_void_p), ("joint_upper", C.c_void_p),
                ("with_base", C.c_int32)]


class PlanDesc(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("n_q", C.c_int32), ("q_joint_ids", C.c_void_p),
                ("n_out", C.c_int32), ("out_link_ids", C.c_void_p),
                ("jac_link_id", C.c_int32), ("n_jac", C.c_int32), ("jac_joint_ids", C.c_void_p),
                ("jac_flags", C.c_uint32)]


class CollDesc(C.Structure):
    _fields_ = [("dtype", C.c_int32), ("n_q", C.c_int32), ("q_joint_ids", C.c_void_p),
                ("n_spheres", C.c_int32), ("sphere_link_ids", C.c_void_p), ("centers", C.c_void_p),
                ("radii", C.c_void_p)]


class IkParams(C.Structure):
    _fields_ = [("max_iters", C.c_int32), ("lam", C.c_double), ("tol_pos", C.c_double),
                ("tol_rot", C.c_double), ("max_step", C.c_double), ("with_rot", C.c_int32),
                ("restarts", C.c_int32), ("seed", C.c_uint64), ("lanes", C.c_int32), ("index_base", C.c_int64),
                ("damp_err", C.c_double)]


class IkSchedStats(C.Structure):
    _fields_ = [("two_phase_calls", C.c_uint64), ("set_waits", C.c_uint64), ("busy_waits", C.c_uint64),
                ("one_phase_fallbacks", C.c_uint64), ("captured_calls", C.c_uint64),
                ("captured_one_phase", C.c_uint64)]


class IkCollParams(C.Structure):
    _fields_ = [("margin", C.c_double), ("band", C.c_double), ("weight", C.c_double), ("feas", C.c_double)]


_lib = None


def lib():
    """Load libkinhip.so (raises if it was not built -- no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    L = C.CDLL(LIB_PATH)
    P, I32, I64, U32, SZ = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_size_t
    sig = {
        "kin_abi_version": ([], C.c_int),
        "kin_last_error": ([], C.c_char_p),
        "kin_limits": ([P, P, P], C.c_int),
        "kin_model_create": ([P, P], C.c_int),
        "kin_model_destroy": ([P], C.c_int),
        "kin_model_num_links": ([P, P], C.c_int),
        "kin_model_num_joints": ([P, P], C.c_int),
        "kin_model_set_angles": ([P, P], C.c_int),
        "kin_model_is_relevant": ([P, I32, I32, P], C.c_int),
        "kin_model_add_link": ([P, I32, P, P], C.c_int),
        "kin_urdf_parse_file": ([C.c_char_p, P], C.c_int),
        "kin_urdf_parse_string": ([C.c_char_p, SZ, P], C.c_int),
        "kin_urdf_destroy": ([P], C.c_int),
        "kin_urdf_tree": ([P, I32, P], C.c_int),
        "kin_urdf_link_name": ([P, I32, P], C.c_int),
        "kin_urdf_joint_name": ([P, I32, P], C.c_int),
        "kin_urdf_find_link": ([P, C.c_char_p, P], C.c_int),
        "kin_urdf_find_joint": ([P, C.c_char_p, P], C.c_int),
        "kin_urdf_link_box": ([P, I32, P, P, P], C.c_int),
        "kin_plan_create": ([P, P, P], C.c_int),
        "kin_plan_destroy": ([P], C.c_int),
        "kin_plan_shape": ([P, P, P, P], C.c_int),
        "kin_plan_run": ([P, P, I64, I64, P, I64, P, I64, P], C.c_int),
        "kin_plan_specialize": ([P, U32], C.c_int),
        "kin_plan_specialized": ([P, P], C.c_int),
        "kin_jit_selfcheck": ([], C.c_int),
        "kin_plan_run_tiled": ([P, I64, P, I64, I64, I64, P, I64, I64, P, I64, I64, P], C.c_int),
        "kin_get_transform_batch": ([P, I32, I32, P, P, I64, I64, I32, P, P, I64, P], C.c_int),
        "kin_get_jacobian_batch": ([P, I32, I32, I32, P, U32, P, I64, I64, P, I64, P, I64, P], C.c_int),
        "kin_ik_dls_batch": ([P, P, P, I64, P, I64, I64, P, P, I64, P], C.c_int),
        "kin_ik_dls_batch_from": ([P, P, P, I64, P, P, I64, I64, P, P, I64, P], C.c_int),
        "kin_ik_dls_batch_trace": ([P, P, P, I64, P, P, I64, I64, P, P, I64, P], C.c_int),
        "kin_point_ik_nakamura_batch": ([P, P, I64, P, I64, I64, P], C.c_int),
        "kin_sdf_create_boxes": ([I32, P, P, P], C.c_int),
        "kin_sdf_destroy": ([P], C.c_int),
        "kin_coll_plan_create": ([P, P, P], C.c_int),
        "kin_coll_batch": ([P, P, C.c_double, P, I64, I64, P, I64, P, I64, P, P], C.c_int),
        "kin_ineq_const_batch": ([P, P, C.c_double, P, I64, I64, P, I64, P, I64, P], C.c_int),
        "kin_pose_const_batch": ([P, P, I64, P, I64, I64, P, I64, P, I64, P, I64, P], C.c_int),
        "kin_coll_ik_plan_create": ([P, P, I32, P], C.c_int),
        "kin_sdf_create_attached": ([P, I32, P, I32, P, P, P, P], C.c_int),
        "kin_coll_batch_scene": ([P, P, C.c_double, P, I64, P, I64, I64, P, I64, P, I64, P, P], C.c_int),
        "kin_ik_coll_batch": ([P, P, P, P, P, I64, P, P, I64, I64, P, P, I64, P], C.c_int),
        "kin_ik_coll_batch_scene": ([P, P, P, P, P, I64, P, I64, P, P, I64, I64, P, P, I64, P], C.c_int),
        "kin_ik_coll_batch_alt": ([P, P, P, P, P, I64, P, I64, P, P, P, I64, I64, P, P, I64, P], C.c_int),
        "kin_plan_ik_sched_stats": ([P, P], C.c_int),
        "kin_plan_specialize_scene": ([P, P], C.c_int),
    }
    # KINHIP_LIB may name a tools-only build (tools/ab.py); KINHIP_SKIP_ABI_CHECK=1 is the explicit opt-out
    # for builds of older sources (tools/ikc_fault_probe.py) that lack newer entry points
    skip_abi = os.environ.get("KINHIP_SKIP_ABI_CHECK") == "1"
    for name, (args, res) in sig.items():
        if skip_abi and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    if not skip_abi and L.kin_abi_version() != ABI_VERSION:
        raise KinError(KIN_E_INVALID, f"{LIB_PATH}: C-ABI version {L.kin_abi_version()}, this binding needs "
                                      f"{ABI_VERSION} (kin_ik_params layout); rebuild the library")
    _lib = L
    return L


def check(rc):
    if rc != KIN_OK:
        msg = lib().kin_last_error()
        raise KinError(rc, msg.decode() if msg else "")
    return rc


def error_class(rc):
    """Map a status to the Python exception the reference's Julia error becomes."""
    return {KIN_E_KEY: KeyError, KIN_E_METHOD: TypeError, KIN_E_PARSE: ValueError}.get(rc, KinError)
