// kinhip_prog.h -- staged evaluation program shared by the host stager
// (kinhip_host.cpp) and the gfx950 kernels (kinhip_fk.hip, kinhip_ik.hip, kinhip_coll.hip).
//
// A plan compiles the reference's per-link transform chain
// (src/algorithm.jl:6-37 + joint_transform, src/mechanism.jl:90-103) into a
// short list of steps.  Every step is
//
//     C <- C_src * F                     (3x4 rigid product, F staged on host)
//     [record o = C.t, z = scale * C.col2]   (pre-motion world joint axis,
//                                              src/algorithm.jl:42-54)
//     C <- C * Rz(theta(q))  or  C <- C * Tz(scale * q)       (joint motion)
//     [output  L = C * X]  [save C to an LDS slot]
//
// "Canonical" frames: the host folds a rotation A (A e_z = joint axis) into F
// so that every moving joint turns about / slides along local z; X = A^T (and,
// for joints held at a constant angle, their motion) restores the link frame
// L of the reference.  Static chains (fixed joints and joints not driven by a
// batch column, at m.angles) are pre-multiplied on the host in fp64 exactly
// like joint_transform does it (quaternion path, `angle == 0.0` shortcut).
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#else
using __hip_internal::int32_t;  // hiprtc's fixed-width types
using __hip_internal::int64_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
#endif

namespace kinhip {

enum : int32_t { MOT_NONE = 0, MOT_REV = 1, MOT_PRISM = 2 };
enum : int32_t { SF_REC = 1, SF_HAS_X = 2, SF_SCALE = 4 };
enum : int32_t { LOAD_NONE = -1, LOAD_ROOT = -2 };
enum : int32_t { PF_JAC = 1, PF_WITH_ROT = 2, PF_RPY = 4, PF_ZERO = 8, PF_BASE = 16 };

// Launches are split into chunks of kChunk configurations so that every lane
// byte offset (uint32, ld_soa / st_soa) fits in 32 bits; chunks are pointer
// offsets into the same SoA arrays (the leading dimensions do not change).
// The IK kernels take kIkChunk per launch.
constexpr int64_t kChunk = int64_t(1) << 27;
constexpr int64_t kIkChunk = kChunk / 8;
// two-phase IK hand-over rings (IkArgsT, kinhip_ik_dev.h): one per lane of a wave (the phase-2 prefix
// scan), their control words one 128-byte line apart
constexpr int kIkSubRings = 64;
constexpr int kIkCtlStride = 32;

constexpr int kMaxChain = 32;  // phase-A steps (root -> spine link), register resident
constexpr int kMaxJacCols = 64;
constexpr int kMaxSlots = 8;

template <typename T>
struct KStep {
    T F[12];   // row-major 3x4 [R | t]
    T X[12];   // output correction (row-major 3x4), valid with SF_HAS_X
    T scale;   // |axis| (revolute: angle map, prismatic: slide scale, record: z scale)
    T lo, hi;  // joint limits of the driving column (IK clamps)
    T pad0;
    int32_t kind;   // MOT_* applied in the kernel
    int32_t jkind;  // joint type for the Jacobian column (MOT_REV / MOT_PRISM)
    int32_t qcol;   // batch column driving the motion (-1: none)
    int32_t flags;  // SF_*
    int32_t out;    // output index (-1: none)
    int32_t load;   // LOAD_NONE: continue, LOAD_ROOT: root frame, >=0: LDS slot
    int32_t save;   // LDS slot to save C into (-1: none)
    int32_t sph0;   // collision plans: spheres [sph0, sph1) hang off this step's frame
    int32_t sph1;
    int32_t pad1;
    uint64_t colmask;  // Jacobian columns this record feeds (phase A only)
};

// collision sphere (src/collision.jl:39-49): centre in the canonical frame of
// its phase-A step (or the root frame), radius, output index
template <typename T>
struct KSphere {
    T c[3];
    T r;
    int32_t out;   // output row (the caller's sphere order)
    uint32_t anc;  // collision-aware IK programs: the variables moving the sphere (KIkcStep::anc)
    int32_t pad[2];
};

// one BoxSDF of a UnionSDF (src/sdf.jl:48-114): inverse world pose (row-major
// 3x4) and half widths
template <typename T>
struct KBox {
    T inv[12];
    T half[3];
    T pad;
};

// A box whose rotation is a signed axis permutation, as a world-axis-aligned
// box: |R^T (p - t)| is a permutation of |p - t|, so the SDF needs only the
// centre and the permuted half widths (kin_sdf_create_boxes sorts these boxes
// first and stores them in this compact form after the KBox array).
template <typename T>
struct KAabb {
    T c[3];
    T half[3];
    T pad[2];
};

// Boxes attached to the links of a scene mechanism (kin_sdf_create_attached; src/sdf.jl:14-32,
// 43-46, 82-97: UnionSDF(mech) follows get_transform of each box's link).  Boxes are grouped by the
// scene's moving frame they ride on (the root / planar base, or the child frame of the last batch
// joint on their path); static offsets down to the box are folded into the box records, which are in
// the group frame.  A group's frame is the root (base) frame times its steps: F, then the joint's
// motion about / along `axis` (kind MOT_REV / MOT_PRISM) by scene column qcol, or F alone (MOT_NONE).
template <typename T>
struct KSceneStep {
    T F[12];    // row-major 3x4
    T axis[3];  // unit joint axis
    T pad;
    int32_t kind;
    int32_t qcol;
    int32_t pad2[2];
};
struct KSceneGroup {
    int32_t step0, step1;  // [step0, step1) of the KSceneStep array
    int32_t box0;          // first box of the group in the KBox array (its KAabb entries at aabb0)
    int32_t na, nb;        // axis-aligned boxes (first), all boxes
    int32_t aabb0;
    int32_t pad[2];
    float bc[3], bh[3];    // the group frame's box enclosing all its boxes (rounded outward): a lower
                           // bound of the group's distance (scene_union's exact cull)
    int32_t pad2[2];
};
constexpr int kMaxSceneGroups = 4;  // moving frames carrying boxes (per-lane frames in registers)

// ---- collision-aware IK program (kin_coll_ik_plan_create, k_ik_tree, kinhip_ikt_dev.h) ----
// The needed kinematic tree -- every moving joint above the target link or above a sphere link, in
// depth-first order -- as one step per moving joint:
//     C <- C_parent * F;  record z = scale * C e_z, m = z x C.t (pre-motion world joint axis, origin);
//     C <- C * motion(q[var]);  [save C to slot `save`]
// C_parent is the previous step's frame (parent == kIkcPrev), the root / planar-base frame
// (kIkcRoot), or a saved branch frame (slot parent >= 0).  Static chains (fixed joints, joints held at
// m.angles) are folded into F on the host in fp64 as joint_transform does (src/mechanism.jl:90-103);
// frames are canonical (the joint axis on local z) as in KStep.  Spheres hang off a step's
// post-motion frame (or the root frame); the target link's frame is frame(tgt_step) * Xt.
constexpr int kIkcMaxVars = 24;   // q columns + 3 base columns (normal equations in registers; PR2: 14 + 3)
constexpr int kIkcMaxSteps = 32;  // moving joints on the needed tree
constexpr int kIkcMaxSlots = 2;   // saved branch frames live at once
constexpr int kIkcMaxSpheres = 64;
constexpr int32_t kIkcPrev = -1, kIkcRoot = -2;
template <typename T>
struct KIkcStep {
    T F[12];   // row-major 3x4
    T scale;   // |axis| (revolute angle map / prismatic slide / record scale)
    T pad[3];
    int32_t kind;    // MOT_REV / MOT_PRISM
    int32_t flags;   // SF_SCALE
    int32_t var;     // variable (q column) driving the joint
    int32_t parent;  // kIkcPrev, kIkcRoot or a slot
    int32_t save;    // slot receiving the post-motion frame (-1: none)
    int32_t sph0, sph1;  // spheres [sph0, sph1) on the post-motion frame
    uint32_t anc;    // variables moving this frame: the joints above it (and itself), the base
};
template <typename T>
struct KIkcProg {
    int32_t nS;         // steps
    int32_t nv;         // variables: n_q joint columns, then base x, y, theta (base_col) if with_base
    int32_t n_q;
    int32_t base_col;   // -1: no planar base
    int32_t n_sph;
    int32_t sph_root0, sph_root1;  // spheres on the root (base) frame
    int32_t tgt_step;   // step whose frame carries the target link (kIkcRoot: the root frame)
    int32_t has_xt;
    uint32_t tgt_mask;  // variables moving the target link (pose Jacobian columns)
    uint32_t free_mask; // variables the solver moves (they move the target or a sphere)
    uint32_t joint_mask;  // variables that are joints (a step records them)
    uint32_t prism_mask;  // joint variables that slide (prismatic Jacobian column)
    int32_t pad;
    T Xt[12];           // target link frame = frame(tgt_step) * Xt
    T vlo[kIkcMaxVars], vhi[kIkcMaxVars];  // joint limits of the variables (base: +-inf)
    // structure of the normal equations: bit c of nzrow[v] (c <= v) is set when entry (v, c) can be nonzero --
    // v and c both move the target link or both move one sphere (every other entry is exactly 0)
    uint32_t nzrow[kIkcMaxVars];
};

// kernel-side tiling: workgroup b works on tile b / tile_blocks (0xffffffff: plain SoA)
struct Tiling {
    uint32_t tile_blocks;
    int64_t tsq, tsp, tsj;  // k_fk: q, poses, jac; k_coll: q, dists, grads
    int64_t tsm;            // k_coll: min_dist
};

struct CollArgs {
    double truncation;
    double offset;    // subtracted from every reported distance (IneqConst margin)
    int32_t n_boxes;  // KBox array (sorted: the first n_aabb are axis-aligned)
    int32_t n_aabb;   // KAabb array placed right after the KBox array
    int32_t accumulate;  // min_dist = min(min_dist, this launch's minimum) (multi-chain plans)
    int32_t pad;
    double bc[3], bh[3];  // world-aligned box enclosing the union: centre, half extents (broad phase)
};

template <typename T>
struct KProg {
    int32_t nA;        // phase-A steps (root -> spine link, padded to the kernel's MAXA)
    int32_t nS;        // total steps
    int32_t n_slots;
    int32_t rows;      // Jacobian rows (3 or 6)
    int32_t n_jac;     // Jacobian columns before the base columns
    int32_t flags;     // PF_*
    int32_t base_col;  // q column of base x (PF_BASE)
    int32_t last_has_x;
    int32_t spine_out;  // output index of the spine link written after phase A (-1: none)
    int32_t pad;
    int32_t n_sph;      // collision plans
    int32_t sph_root0, sph_root1;  // spheres on the root frame
    int32_t pad2;
    uint64_t zmask;    // irrelevant Jacobian columns (zero-filled with PF_ZERO)
    T Xlast[12];       // spine link frame = C(after phase A) * Xlast
};

}  // namespace kinhip
