"""kinhip -- MI355X-native batched kinematics (FK, Jacobian, IK) for Kinematics.jl users.

Python host mirror of the reference's API over the C-ABI library
``libkinhip.so`` (include/kinhip.h).  The compute path is the gfx950 HIP
engine only; importing this package on a machine without the built library
fails loudly.
"""
from ._lib import (  # noqa: F401
    KIN_SPEC_COLL, KIN_SPEC_FK, KIN_SPEC_IK, KIN_SPEC_IK_COLL, KIN_SPEC_IK_COLL_SCENE, KIN_SPEC_NAKAMURA, KinError, LIB_PATH,
    lib,
)
from .mechanism import (  # noqa: F401
    BoxMetaData, Joint, Link, Mechanism, Plan, SphereMetaData, Transform, add_new_link, child_joints, child_link,
    child_links, find_joint, find_link, get_jacobian, get_jacobian_, get_jacobian_batch, get_joint_angles,
    get_joint_angles_, get_transform, get_transform_batch, inverse_kinematics_, is_relevant, isleaf, isroot,
    joint_angle, parent_joint, parent_link, parse_urdf, point_inverse_kinematics_nakamura, rotation, rpy,
    set_joint_angle, set_joint_angles, tiled, translation, untiled,
)
from .synth import uniform_configs  # noqa: F401
from .collision import (  # noqa: F401
    FETCH_ARM_SPHERES, FETCH_LINK_SPHERES, PR2_ARM_SPHERES, PR2_LARM_JOINTS, PR2_MANIP_POSE, PR2_RARM_JOINTS,
    AttachedUnionSDF, BoxSDF, CollisionIKPlan, CollisionPlan, SweptSphereCollisionChecker, UnionSDF,
    add_coll_links, add_fetch_arm_spheres, compute_coll_dists, compute_coll_dists_, compute_coll_dists_and_grads,
    compute_coll_dists_and_grads_, compute_swept_sphere, fridge_sdf,
)
from .planning import (  # noqa: F401
    ConfigurationConstraint, EqConst, IneqConst, Objective, PoseConstraint, construct_problem,
    collision_aware_ik, create_straight_trajectory, plan_trajectory,
)

FETCH_ARM_JOINTS = [
    "torso_lift_joint", "shoulder_pan_joint", "shoulder_lift_joint", "upperarm_roll_joint",
    "elbow_flex_joint", "forearm_roll_joint", "wrist_flex_joint", "wrist_roll_joint",
]
