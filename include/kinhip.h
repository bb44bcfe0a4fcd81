/*
 * kinhip.h -- C-ABI of the MI355X batched kinematics engine (libkinhip.so).
 *
 * Drop-in boundary for Kinematics.jl's hot path.  The reference has no FFI
 * layer (it is pure Julia); these entry points are what a Julia `ccall` shim
 * (kinematics.jl_amd/julia/KinematicsHIP.jl) binds in place of
 * the Julia methods cited on each declaration.  Plain C types only: device
 * pointers and sizes in, status codes out, never an exception.
 *
 * Conventions
 *  - Link / joint ids are 1-based, exactly `link.id` / `joint.id` of the
 *    reference (ids follow URDF document order, src/load_urdf.jl:22-32).
 *  - Transforms crossing the boundary on the host are 4x4 column-major
 *    (`Transform.mat`, src/transform.jl:3-5).
 *  - Batched device arrays are structure-of-arrays with the configuration
 *    index fastest = Julia column-major `Matrix{T}(N, k)` / `Array{T,3}(N, r, c)`,
 *    so `pointer(A)` passes zero-copy:
 *      q      : column c at q[c*ldq + i]; columns = the plan's q joints in order,
 *               then (x, y, theta) if the model was created with_base.
 *      poses  : [n_out][12][ldp]; the 12 values are the 3x4 column-major top of
 *               the 4x4 (R11 R21 R31 R12 R22 R32 R13 R23 R33 tx ty tz).
 *      jac    : [n_cols][rows][ldj]; rows = 6 (with_rot) or 3; n_cols = n_jac
 *               (+3 base columns if with_base) -- get_jacobian!'s mat_out.
 *  - dtype selects float (KIN_F32) or double (KIN_F64) for every batched array
 *    of one call.  Host-side tree data is always double.
 *  - Every batched call is asynchronous on the given hipStream_t (passed as
 *    void*; NULL = the null stream) and capture-safe (no allocation, copy or
 *    synchronisation inside), with one exception: the first kin_ik_dls_batch
 *    call of a plan that may use the two-phase schedule (restarts > 0, lanes = 0,
 *    <= 2^20 targets) allocates that plan's scratch (synchronising; make it once
 *    outside a stream capture).
 *  - Errors: a negative kin_status; kin_last_error() returns a thread-local
 *    message.  Reference exceptions map to: KeyError -> KIN_E_KEY,
 *    MethodError (Jacobian column of a fixed joint) -> KIN_E_METHOD,
 *    throw(Exception) on an unknown URDF joint type -> KIN_E_PARSE.
 *  - Thread safety: models/plans are immutable after creation except through
 *    kin_model_set_angles / kin_model_add_link (not concurrent with use).
 *    Distinct streams may run plans concurrently from different host threads.
 *  - Devices: a plan / kin_sdf belongs to the HIP device that was current when
 *    it was created.  Every run / specialise call checks the current device
 *    and returns KIN_E_INVALID on a mismatch (one plan per device for
 *    multi-GPU callers); kin_get_*_batch keep one cached plan per device.
 */
#ifndef KINHIP_H
#define KINHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KINHIP_API __attribute__((visibility("default")))
/* ABI version (kin_abi_version): 2 since kin_ik_params gained damp_err (round 4) -- a caller built against
 * version 1 passes a shorter kin_ik_params, so every binding checks kin_abi_version() == KINHIP_ABI_VERSION
 * before its first call (the Python mirror, the Julia shim and examples/kin_c_demo.c refuse a mismatch;
 * INTEGRATION.md). */
#define KINHIP_ABI_VERSION 2

typedef enum {
    KIN_OK = 0,
    KIN_E_INVALID = -1,     /* bad argument / malformed tree */
    KIN_E_KEY = -2,         /* unknown link / joint id or name (Julia KeyError) */
    KIN_E_METHOD = -3,      /* no method (Jacobian column of a relevant fixed joint) */
    KIN_E_DEVICE = -4,      /* HIP runtime error */
    KIN_E_UNSUPPORTED = -5, /* outside the engine's limits (see kin_limits) */
    KIN_E_NOMEM = -6,
    KIN_E_PARSE = -7,       /* URDF parse error / unsupported joint type */
    KIN_E_IO = -8
} kin_status;

typedef enum { KIN_F32 = 0, KIN_F64 = 1 } kin_dtype;

enum { KIN_JOINT_FIXED = 0, KIN_JOINT_REVOLUTE = 1, KIN_JOINT_PRISMATIC = 2 };

/* get_jacobian! keyword/positional flags (src/algorithm.jl:83-88) */
enum {
    KIN_WITH_ROT = 1u,  /* rows 4:6 present (with_rot) */
    KIN_RPY_JAC = 2u,   /* rows 4:6 are d(rpy)/dt (rpy_jac=true) */
    KIN_ZERO_FILL = 4u  /* get_jacobian (zeros) instead of get_jacobian! (untouched) */
};

/* ------------------------------------------------------------------------- */
/* Library                                                                    */
/* ------------------------------------------------------------------------- */
KINHIP_API int kin_abi_version(void);
KINHIP_API const char* kin_last_error(void);
/* Engine limits: max phase-A chain steps, max Jacobian columns, max outputs. */
KINHIP_API int kin_limits(int32_t* max_chain, int32_t* max_jac_cols, int32_t* max_slots);

/* ------------------------------------------------------------------------- */
/* Model = the kinematic tree of a Mechanism (src/mechanism.jl:147-181)       */
/* ------------------------------------------------------------------------- */
typedef struct kin_tree_desc {
    int32_t n_links;
    int32_t n_joints;
    const int32_t* joint_type;  /* [n_joints] KIN_JOINT_* (continuous = revolute) */
    const int32_t* joint_plink; /* [n_joints] 1-based parent link id */
    const int32_t* joint_clink; /* [n_joints] 1-based child link id */
    const double* joint_pose;   /* [n_joints][16] 4x4 column-major (Joint.pose) */
    const double* joint_axis;   /* [n_joints][3]  (Revolute/Prismatic .axis) */
    const double* joint_lower;  /* [n_joints] or NULL (= -Inf) */
    const double* joint_upper;  /* [n_joints] or NULL (= +Inf) */
    int32_t with_base;          /* Mechanism.with_base: planar base (x, y, theta) */
} kin_tree_desc;

typedef struct kin_model kin_model;

/* Mechanism(...) constructor + create_rptable: src/mechanism.jl:117-139, 166-181.
 * Stages nothing on the device yet (plans do). */
KINHIP_API int kin_model_create(const kin_tree_desc* desc, kin_model** out);
KINHIP_API int kin_model_destroy(kin_model* m);
KINHIP_API int kin_model_num_links(const kin_model* m, int32_t* out);
KINHIP_API int kin_model_num_joints(const kin_model* m, int32_t* out);
/* m.angles for joints NOT driven by a batch column (set_joint_angle(s),
 * src/mechanism.jl:199-231).  angles: [n_joints] or NULL (zeros). Plans created
 * afterwards bake these values in; existing plans keep theirs. */
KINHIP_API int kin_model_set_angles(kin_model* m, const double* angles);
/* is_relevant(m, joint, link): src/mechanism.jl:277 */
KINHIP_API int kin_model_is_relevant(const kin_model* m, int32_t joint_id, int32_t link_id, int32_t* out);
/* add_new_link(m, new_link, parent, pose): src/mechanism.jl:238-267.
 * Appends a link and a fixed joint named after it; returns the new link id. */
KINHIP_API int kin_model_add_link(kin_model* m, int32_t parent_link_id, const double* pose16,
                                  int32_t* new_link_id);

/* ------------------------------------------------------------------------- */
/* URDF (host; replaces parse_urdf's skrobot call, src/load_urdf.jl:20-80)     */
/* ------------------------------------------------------------------------- */
typedef struct kin_urdf kin_urdf;
KINHIP_API int kin_urdf_parse_file(const char* path, kin_urdf** out);
KINHIP_API int kin_urdf_parse_string(const char* xml, size_t len, kin_urdf** out);
KINHIP_API int kin_urdf_destroy(kin_urdf* u);
/* Tree of the parsed URDF; the pointers stay valid for the lifetime of u.
 * with_base is copied into desc->with_base. */
KINHIP_API int kin_urdf_tree(const kin_urdf* u, int32_t with_base, kin_tree_desc* desc);
KINHIP_API int kin_urdf_link_name(const kin_urdf* u, int32_t link_id, const char** name);
KINHIP_API int kin_urdf_joint_name(const kin_urdf* u, int32_t joint_id, const char** name);
/* find_link / find_joint (src/mechanism.jl:191-192); KIN_E_KEY if absent */
KINHIP_API int kin_urdf_find_link(const kin_urdf* u, const char* name, int32_t* id);
KINHIP_API int kin_urdf_find_joint(const kin_urdf* u, const char* name, int32_t* id);
/* BoxMetaData of a link's collision geometry (src/load_urdf.jl:1-18).
 * *has_box = 0 when the link has no box collision. */
KINHIP_API int kin_urdf_link_box(const kin_urdf* u, int32_t link_id, int32_t* has_box,
                                 double* extents3, double* origin16);

/* ------------------------------------------------------------------------- */
/* Plans: one staged, device-resident evaluation program per request          */
/* ------------------------------------------------------------------------- */
typedef struct kin_plan_desc {
    int32_t dtype;               /* kin_dtype */
    int32_t n_q;                 /* batch columns: set_joint_angles(m, joints, angles) */
    const int32_t* q_joint_ids;
    int32_t n_out;               /* get_transform(m, link) for each of these links */
    const int32_t* out_link_ids;
    int32_t jac_link_id;         /* get_jacobian!(m, link, joints, ...); 0 = none */
    int32_t n_jac;
    const int32_t* jac_joint_ids;
    uint32_t jac_flags;          /* KIN_WITH_ROT | KIN_RPY_JAC | KIN_ZERO_FILL */
} kin_plan_desc;

typedef struct kin_plan kin_plan;

/* Stages the tree for this request onto the current HIP device
 * (synchronous; call outside stream capture). */
KINHIP_API int kin_plan_create(const kin_model* m, const kin_plan_desc* desc, kin_plan** out);
KINHIP_API int kin_plan_destroy(kin_plan* p);
/* Number of batch columns q must hold, Jacobian rows and columns. */
KINHIP_API int kin_plan_shape(const kin_plan* p, int32_t* n_qcols, int32_t* jac_rows, int32_t* jac_cols);

/* Batched get_transform (+ get_jacobian!) for N configurations:
 * src/algorithm.jl:1-21 and :83-106 with set_joint_angles per config.
 * poses may be NULL when n_out == 0; jac may be NULL when the plan has no
 * Jacobian.  Device pointers; async on stream. */
KINHIP_API int kin_plan_run(const kin_plan* p, const void* q, int64_t ldq, int64_t n,
                            void* poses, int64_t ldp, void* jac, int64_t ldj, void* stream);

/* Tiled structure-of-arrays variant of kin_plan_run (the MI355X-preferred
 * layout for large batches): configurations are grouped in
 * tiles of `tile` (a multiple of 256, <= 2^26); element (config i, row r) of an
 * array X lives at X[(i / tile) * ts + r * ld + (i % tile)], i.e. a Julia
 * Array{T,3}(ld, rows, ntiles) with ld >= tile and ts >= rows * ld (the last
 * tile may be partial).  tile >= n is exactly kin_plan_run.  Each workgroup
 * then writes one contiguous tile-row run per output row instead of 60 streams
 * 4 MB apart (profiles/r01_tile_probe.txt: +10% HBM rate for FK + J). */
KINHIP_API int kin_plan_run_tiled(const kin_plan* p, int64_t tile, const void* q, int64_t ldq, int64_t tsq, int64_t n,
                                  void* poses, int64_t ldp, int64_t tsp, void* jac, int64_t ldj, int64_t tsj,
                                  void* stream);

/* Plan specialisation: compiles this plan's staged program at run time
 * (hiprtc, gfx950) into kernels in which every fixed transform coefficient,
 * joint kind, output index and Jacobian column is a compile-time constant --
 * zero terms of the 3x4 products vanish and each joint's motion is chosen
 * statically.  Afterwards the plan's launches of the selected kernels use the
 * specialised code.  `kernels` is a mask of KIN_SPEC_* (0 = every kind that
 * applies to the plan).  Synchronous (seconds on first use; code objects are
 * cached per process by program text); call outside stream capture.  FK,
 * Jacobian and collision results equal the generic kernels' for finite inputs
 * (up to the sign of zeros); iterative IK may differ in the last bits where
 * the two compilations contract a product-sum differently.
 * KIN_E_DEVICE (message from hiprtc) leaves the plan on its generic kernels. */
enum {
    KIN_SPEC_FK = 1u,        /* kin_plan_run(_tiled), kin_pose_const_batch (not the one-shot kin_get_*_batch) */
    KIN_SPEC_IK = 2u,        /* kin_ik_dls_batch (with_rot 0/1, every lane count) */
    KIN_SPEC_NAKAMURA = 4u,  /* kin_point_ik_nakamura_batch */
    KIN_SPEC_COLL = 8u,      /* kin_coll_batch, kin_ineq_const_batch (spheres folded; boxes stay data) */
    KIN_SPEC_IK_COLL = 16u,  /* kin_ik_coll_batch (plans of kin_coll_ik_plan_create) */
    KIN_SPEC_IK_COLL_SCENE = 32u  /* kin_ik_coll_batch_scene over unions of <= 2 moving scene groups (the
                                     scene's frames and boxes stay launch data: one code object per plan) */
};
KINHIP_API int kin_plan_specialize(kin_plan* p, uint32_t kernels);
/* The KIN_SPEC_* mask the plan currently runs specialised. */
KINHIP_API int kin_plan_specialized(const kin_plan* p, uint32_t* kernels);
/* Compiles (does not load) a synthetic program with every specialised kernel kind in
 * both precisions: checks run-time compilation on the host, no GPU needed.  0 = ok;
 * otherwise kin_last_error() holds the compiler log. */
KINHIP_API int kin_jit_selfcheck(void);

/* One-shot conveniences with an internal per-model plan cache (the first call
 * for a request stages it synchronously; later calls are async).
 * kin_get_transform_batch: poses of n_out links.  kin_get_jacobian_batch: the
 * Jacobian of link over jac joints (pose optional).  The q columns are the
 * given joints (+ base). */
KINHIP_API int kin_get_transform_batch(kin_model* m, int32_t dtype, int32_t n_q, const int32_t* q_joint_ids,
                                       const void* q, int64_t ldq, int64_t n, int32_t n_out,
                                       const int32_t* out_link_ids, void* poses, int64_t ldp, void* stream);
KINHIP_API int kin_get_jacobian_batch(kin_model* m, int32_t dtype, int32_t link_id, int32_t n_joints,
                                      const int32_t* joint_ids, uint32_t jac_flags, const void* q,
                                      int64_t ldq, int64_t n, void* pose, int64_t ldp, void* jac,
                                      int64_t ldj, void* stream);

/* ------------------------------------------------------------------------- */
/* Inverse kinematics                                                          */
/* ------------------------------------------------------------------------- */
/* Damped-least-squares IK (build-defined batched replacement of the SLSQP loop
 * of inverse_kinematics!, src/inverse_kinematics.jl:23-64; iterates unpinned,
 * acceptance pinned by test/test_inverse_kinematics.jl:19-23).
 * The plan must have a Jacobian whose joints equal its q joints (same order)
 * and jac_flags without KIN_RPY_JAC; its jac link is the IK target link.
 *   target : [12][ldt] target poses (3x4 column-major)
 *   q      : [n_qcols][ldq] initial angles in, solution out (clamped to limits)
 *   iters  : [n] int32 or NULL: the iterations the converged attempt used (0..max_iters, so a target
 *            converging at exactly max_iters reports max_iters), max_iters + 1 if no attempt converged
 *   err    : [2][n] final |dp|, |rot err| (dtype) or NULL
 * Precision: fp64 uses exact arithmetic throughout (its iterates match the CPU
 * restatement); fp32 uses the hardware sin / cos / rsqrt / rcp / sqrt and a
 * polynomial atan2 (~1e-7..4e-7 error) inside the iteration -- the result is still checked against tol_pos /
 * tol_rot by the same iteration.                                                 */
typedef struct kin_ik_params {
    int32_t max_iters;  /* e.g. 64 */
    double lambda;      /* damping, e.g. 1e-2.  0 is the undamped Gauss-Newton step: at a singular arm (Fetch at
                           q = 0) its normal equations are singular and a target can end on NaN angles (iters =
                           max_iters + 1), in fp64 as in the oracle.  The fp32 kernels solve the damped system in
                           fp32 only for lambda^2 >= 0.99e-4 (and not in attempt 0's first 3 iterations), in fp64
                           otherwise */
    double tol_pos;     /* |dp| tolerance, e.g. 1e-3 */
    double tol_rot;     /* |axis-angle error| tolerance, e.g. 1e-3 */
    double max_step;    /* max |dq|_inf per iteration, e.g. 0.5 */
    int32_t with_rot;   /* 0: position only; 1: residual [p* - p; log(R* R^T)] (axis-angle) with the geometric
                           Jacobian; 2: the reference's f_objective (src/inverse_kinematics.jl:38-50): residual
                           [p* - p; rpy(target) - rpy(pose)] (angle differences wrapped to (-pi, pi]) with the
                           rpy_jac=true Jacobian, converged when |dp| < tol_pos and |d rpy| < tol_rot (err row 1
                           is then |d rpy|).  The wrap deviates from the reference on purpose: its raw difference
                           is ~2 pi when the two yaws (or rolls) lie on either side of +-pi, which sends the arm
                           the long way round; tests/test_gpu_ik_rpy.py::test_rpy_difference_wraps_at_pi */
    int32_t restarts;   /* 0: none; else max_iters is split into restarts+1 attempts and each new
                           attempt re-draws the relevant joints uniformly within their limits
                           (U[-pi, pi] if unbounded) from a counter hash of (seed, i, attempt, column) */
    uint64_t seed;
    int32_t lanes;      /* lanes per target running attempts side by side: 0 = auto, else 1/2/4/8.
                           Results are identical for every value (each attempt's arithmetic is the
                           sequential schedule's); only the parallelism changes.  With 0 and restarts,
                           batches of more than one round of waves (up to 2^20 targets) run in two
                           launches: attempt 0 of every target, then the remaining attempts of the
                           targets attempt 0 did not solve, side by side (same results; a batch of one
                           round hands attempt 0 over after 5/8 of its iterations and phase 2 resumes it
                           beside the others, bit for bit).  The two-phase scratch (first call:
                           hipMalloc of 8 sets of ~16 MiB, 64 hand-over rings each, synchronising) is
                           per plan: an eager call takes one of 4 sets, ordered after the set's previous
                           call by stream order (same stream) or, when that call is still in flight on
                           another stream, by a host wait on its event, so calls from any thread, stream or
                           handle (hipStreamPerThread included) never share a set in flight; the set its
                           stream used last is preferred, else one that has finished, else the least
                           recently used (kin_plan_ik_sched_stats counts the waits).  A captured graph
                           keeps the set of its captured call. */
    int64_t index_base; /* global index of target 0 in the restart draws' hash: a caller that shards one
                           target set across processes passes its shard's offset, so every target gets
                           the same draws (and results) as in a single process; 0 otherwise */
    double damp_err;    /* error-scaled damping (Levenberg-Marquardt after Sugihara): each iteration solves with
                           lambda^2 + damp_err * (|dp|^2 + |rot|^2) in place of lambda^2 -- heavy damping far from
                           the target, lambda near it.  0: fixed lambda.  kin_ik_dls_batch(_from) only (the
                           collision-aware IK requires 0).  Config 4's headline leg runs 0 (fixed lambda); the
                           bench's config4_ik_dls_damped leg runs 0.01 with max_step 1 (tools/ik_damp_explore.py) */
} kin_ik_params;
KINHIP_API int kin_ik_dls_batch(const kin_plan* p, const kin_ik_params* prm, const void* target, int64_t ldt,
                                void* q, int64_t ldq, int64_t n, int32_t* iters, void* err, int64_t lde,
                                void* stream);
/* kin_ik_dls_batch with the starting angles read from q0 ([n_q][ldq], same leading dimension as q,
 * not modified) instead of q: the chain's columns (and base columns) of q are written for every
 * target without being read, other columns of q are left as they are.  Same results as copying q0
 * into q and calling kin_ik_dls_batch, without the copy; lets a caller solve many target batches
 * from one q0 (the reference's inverse_kinematics! starts from the mechanism's current angles,
 * src/inverse_kinematics.jl:32-64).  q0 == q is the in-place call; other overlaps are not allowed. */
KINHIP_API int kin_ik_dls_batch_from(const kin_plan* p, const kin_ik_params* prm, const void* target, int64_t ldt,
                                     const void* q0, void* q, int64_t ldq, int64_t n, int32_t* iters, void* err,
                                     int64_t lde, void* stream);

/* kin_ik_dls_batch_from that also records the residual of every iterate: trace [2 (max_iters + 1)][ldtr]
 * (dtype) gets |dp| (row 2k) and |rot err| (row 2k + 1) of iterate k = 0, 1, ... as the solver reaches it
 * (rows of iterations a target does not reach are left as they are).  One lane per target (lanes is
 * ignored, attempts in sequence).  This is what the reference's ftol_abs stopping rule needs (NLopt stops
 * when one step changes the objective by less than ftol, src/inverse_kinematics.jl:23-30): one launch of
 * max_iters steps gives every iterate's objective, a second of k steps the stopping iterate -- O(max_iters)
 * steps (kinhip.inverse_kinematics_). */
KINHIP_API int kin_ik_dls_batch_trace(const kin_plan* p, const kin_ik_params* prm, const void* target, int64_t ldt,
                                      const void* q0, void* q, int64_t ldq, int64_t n, int32_t* iters, void* trace,
                                      int64_t ldtr, void* stream);

/* Counters of the plan's two-phase IK scratch-set scheduling (kin_ik_params.lanes above), for tests and
 * diagnostics; no reference counterpart (the reference is single-threaded). */
typedef struct kin_ik_sched_stats {
    uint64_t two_phase_calls;     /* eager calls that took a scratch set (two-phase schedule) */
    uint64_t set_waits;           /* of those, calls that waited on the host for the set's previous call, still
                                     in flight on another stream (or another thread's per-thread stream) */
    uint64_t busy_waits;          /* calls that found every set between take and event record in other
                                     threads and waited (microseconds) for one */
    uint64_t one_phase_fallbacks; /* eager two-phase calls that ran the one-phase schedule for want of a set
                                     (0 by construction since round 6) */
    uint64_t captured_calls;      /* two-phase calls made inside a stream capture that took a graph set */
    uint64_t captured_one_phase;  /* captured two-phase calls that ran one phase (the 4 graph sets taken) */
} kin_ik_sched_stats;
KINHIP_API int kin_plan_ik_sched_stats(const kin_plan* p, kin_ik_sched_stats* out);

/* point_inverse_kinematics_nakamura (src/algorithm.jl:116-131), batched:
 * 50 SR-inverse iterations, `.+ sr_weight` broadcast quirk reproduced.
 * points: [3][ldpt]; q: [n_q][ldq] in/out.  Plan: Jacobian over its q joints,
 * model without base. */
KINHIP_API int kin_point_ik_nakamura_batch(const kin_plan* p, const void* points, int64_t ldpt, void* q,
                                           int64_t ldq, int64_t n, void* stream);

/* ------------------------------------------------------------------------- */
/* Collision: swept spheres vs a union of box SDFs                             */
/* (src/collision.jl:51-103, src/sdf.jl:48-119)           */
/* ------------------------------------------------------------------------- */
typedef struct kin_sdf kin_sdf;
/* UnionSDF of BoxSDF(pose, width) (src/sdf.jl:48-114): box k has world pose
 * poses16[k] (4x4 column-major) and full widths widths3[k].  Uploaded to the
 * current device in both precisions. */
KINHIP_API int kin_sdf_create_boxes(int32_t n_boxes, const double* poses16, const double* widths3, kin_sdf** out);
KINHIP_API int kin_sdf_destroy(kin_sdf* s);

/* UnionSDF(mech) of a scene mechanism (src/sdf.jl:76-97): box k = BoxSDF(origin, width) attached to link
 * link_ids[k] of `scene` (attach_to_link, :43-46), its world pose get_transform(scene, link) * origin
 * (:14-32) -- e.g. the fridge's door box follows door_joint.  The scene joints q_joint_ids (+ the scene's
 * planar base when the scene model has with_base) are inputs of every kin_coll_batch_scene call; other
 * scene joints are held at the scene model's angles (kin_model_set_angles) as of this call.  Boxes ride
 * on at most 4 moving frames (the root / base and the child frames of batch joints).  Uploaded to the
 * current device in both precisions. */
KINHIP_API int kin_sdf_create_attached(const kin_model* scene, int32_t n_q, const int32_t* q_joint_ids,
                                       int32_t n_boxes, const int32_t* link_ids, const double* origins16,
                                       const double* widths3, kin_sdf** out);

typedef struct kin_coll_desc {
    int32_t dtype;
    int32_t n_q;                     /* batch columns (+3 base) and gradient columns */
    const int32_t* q_joint_ids;
    int32_t n_spheres;               /* SweptSphereCollisionChecker.sphere_links (src/collision.jl:32-37) */
    const int32_t* sphere_link_ids;  /* sphere centre = origin of this link ... */
    const double* centers;           /* ... plus this offset in the link frame ([n][3], NULL = 0) */
    const double* radii;             /* [n] */
} kin_coll_desc;
/* Spheres may hang off several moving chains (e.g. both arms, or arm + head): the plan groups them by
 * chain, stages one program per group and launches them in turn (min_dist accumulates); gradient
 * columns of joints off a sphere's chain are 0.  Limits: kin_limits (KIN_E_UNSUPPORTED beyond). */
KINHIP_API int kin_coll_plan_create(const kin_model* m, const kin_coll_desc* desc, kin_plan** out);
/* compute_coll_dists(_and_grads)! for N configurations:
 *   dists    [n_spheres][ldd]       sdf(centre) - radius (or NULL)
 *   grads    [n_spheres][n_q(+3)][ldg]  grad_sdf^T J(3 x n) of each sphere link (or NULL)
 *   min_dist [N]                    min over spheres (or NULL)
 * A sphere farther than `truncation` reports `truncation` and a zero gradient
 * (truncation_dist, src/collision.jl:84-87).  The SDF gradient is analytic
 * (the reference takes a forward difference, eps 1e-7).  fp32 places the
 * spheres with the hardware sin / cos (~4e-7 error; fp64 is exact).  With a
 * finite truncation, spheres provably beyond it skip the boxes (same results).
 * Gradient columns of joints that do not move a sphere are 0.  (Deliberate
 * difference: the reference allocates its 3 x n_dof `jac` once outside the
 * sphere loop, src/collision.jl:76, and get_jacobian! writes only the columns
 * relevant to each sphere's link, so a sphere that follows one on a deeper
 * link inherits that sphere's columns; the zeros here are the true
 * derivative.  Parity for such mixed-link sphere orders is therefore pinned
 * against the finite-difference truth, not the reference's buffer.) */
KINHIP_API int kin_coll_batch(const kin_plan* p, const kin_sdf* sdf, double truncation, const void* q, int64_t ldq,
                              int64_t n, void* dists, int64_t ldd, void* grads, int64_t ldg, void* min_dist,
                              void* stream);
/* (Layout: rows whose leading dimension is a power of two of >= 2^16 elements -- e.g. ld = n = 2^20 -- put a
 * wave's 126 row streams on the same HBM channels; ld = n + 256 runs ~10% faster.  A tiled collision
 * layout was measured and dropped: it lost to padded rows in two driver runs) */

/* kin_coll_batch against boxes attached to a scene (kin_sdf_create_attached): scene_q [n_scene_cols][lds]
 * holds the scene joint values (+ base x, y, theta) of every sample -- one launch sweeps e.g. many door
 * angles -- or, with lds = 0, one set of values for the whole launch.  Plain SoA only.  Plans specialised
 * with KIN_SPEC_COLL run kernels with the arm chain and spheres as constants (the scene's groups, steps
 * and boxes stay launch data) for unions of up to 4 moving groups; the generic kernel otherwise. */
KINHIP_API int kin_coll_batch_scene(const kin_plan* p, const kin_sdf* sdf, double truncation, const void* q,
                                    int64_t ldq, const void* scene_q, int64_t lds, int64_t n, void* dists,
                                    int64_t ldd, void* grads, int64_t ldg, void* min_dist, void* stream);
/* Compiles kin_coll_batch_scene's kernels of plan p (kin_coll_plan_create) with one attached union's
 * tables -- its groups, the scene steps of each group's frame, the boxes -- as constants as well (hiprtc,
 * gfx950; synchronous, cached per process by source).  A planar base and a joint about a coordinate
 * axis then leave a group frame of a few lane values (the fridge: 10 instead of 24 registers) and the
 * boxes' data are immediates.  Later kin_coll_batch_scene calls of p with this sdf run them; results are
 * those of the other kernels (up to the sign of a zero).  The union is identified by the kin_sdf object:
 * a new kin_sdf (even of the same scene) runs the plan's other kernels until it is specialised too.
 * No reference counterpart (the reference evaluates one sphere at a time, src/collision.jl:67-94). */
KINHIP_API int kin_plan_specialize_scene(kin_plan* p, const kin_sdf* sdf);


/* ------------------------------------------------------------------------- */
/* Collision-aware IK: inverse_kinematics!(m, link, joints, target, sscc, sdf;  */
/* use_bistage) (src/inverse_kinematics.jl:1-21), many targets per launch       */
/* ------------------------------------------------------------------------- */
/* An IK plan of `link_id` over the q joints (kin_ik_dls_batch works on it: stage 1 of the bistage
 * solve) with the tree of the target link and every swept sphere staged for kin_ik_coll_batch.  Spheres
 * may hang off any chain of the tree (both arms of a two-arm robot, torso / head links: the reference's
 * fridge_demo.jl scene); the solver's variables are the q joints that move the target link or a sphere
 * (+ the planar base), the other q columns are passed through.  Limits (KIN_E_UNSUPPORTED beyond):
 * q columns + 3 base columns <= 24 (PR2's two arms + base: 17), <= 32 moving joints on the needed tree, <= 64 spheres, at most 2 branch
 * frames live at once.  Zero spheres is the plain pose problem (the reference's own PR2 test builds its
 * checker with none, test/test_inverse_kinematics.jl:63). */
KINHIP_API int kin_coll_ik_plan_create(const kin_model* m, const kin_coll_desc* desc, int32_t link_id, kin_plan** out);

typedef struct kin_ik_coll_params {
    double margin;  /* IneqConst(sscc, joints, sdf, 1, margin): every sphere at least margin from the union
                       (the reference's stage 2 uses 0.02, src/inverse_kinematics.jl:16) */
    double band;    /* spheres with d < margin + band get a penalty row pushing them to margin + band (e.g. 0:
                       rows only for violating spheres; a positive band keeps a clearance) */
    double weight;  /* weight of a sphere row against the pose rows (e.g. 1) */
    double feas;    /* converged only when every sphere has d >= margin - feas (e.g. 1e-6) */
} kin_ik_coll_params;
/* Stage 2 of the bistage solve for N targets (stage 1 = kin_ik_dls_batch_from on the same plan): from
 * q0 ([n_q(+3)][ldq], read; q0 == q is in place) damped Gauss-Newton steps on the pose residual of
 * kin_ik_params.with_rot (2 = the reference's rpy objective) plus one-sided penalty rows
 * a_k = grad sdf^T J_k of the spheres inside the band, normal equations over the free variables,
 * joint limits by an active set and a clamp; restarts as in kin_ik_dls_batch (lambda > 0; every free
 * joint re-drawn).  lanes: 0 = auto (specialised plans: a target's restart attempts side by side in 4
 * lane groups for batches of at most 65,536 targets, its spheres shared out over 16 lanes per group
 * while the batch has at most ~4,096 targets), 1 = one lane per target (attempts in sequence),
 * 2 / 4 / 8 = attempts side by side on one lane each, 16 = spheres over 16 lanes, 64 = both (16 x 4);
 * identical results for every setting (the generic kernel runs 4 attempt groups for lanes 2 / 4 / 8 on
 * trees of <= 12 variables, one lane otherwise).
 * Converged (iters <= max_iters, else max_iters + 1) when |dp| < tol_pos, |rot| < tol_rot and every
 * sphere has d >= margin - feas; a target no attempt solves gets the attempt whose end state has the
 * lowest |dp|^2 + |rot|^2 + weight^2 max(0, margin - min d)^2 (NLopt returns its best point likewise).
 * err: [3][lde] |dp|, |rot err|, min sphere distance of the returned state (or NULL). */
KINHIP_API int kin_ik_coll_batch(const kin_plan* p, const kin_sdf* sdf, const kin_ik_params* prm,
                                 const kin_ik_coll_params* cprm, const void* target, int64_t ldt, const void* q0,
                                 void* q, int64_t ldq, int64_t n, int32_t* iters, void* err, int64_t lde,
                                 void* stream);
/* kin_ik_coll_batch against boxes attached to a scene mechanism (kin_sdf_create_attached; UnionSDF(fridge)
 * of fridge_demo.jl / test/test_inverse_kinematics.jl:52-86): scene_q [n_scene_cols][lds] holds the scene
 * joint values (+ base x, y, theta) of each target -- one launch solves e.g. a reach into the fridge at a
 * different door angle per target -- or, with lds = 0, one set for the whole launch.  The scene stays
 * fixed during a target's solve.  Lanes as kin_ik_coll_batch: plans specialised with
 * KIN_SPEC_IK_COLL_SCENE run the S x G-lane kernels for unions of up to 2 moving groups (the fridge and
 * its door), bit-identical to the generic kernel; wider scenes run the generic kernel. */
KINHIP_API int kin_ik_coll_batch_scene(const kin_plan* p, const kin_sdf* sdf, const kin_ik_params* prm,
                                       const kin_ik_coll_params* cprm, const void* target, int64_t ldt,
                                       const void* scene_q, int64_t lds, const void* q0, void* q, int64_t ldq,
                                       int64_t n, int32_t* iters, void* err, int64_t lde, void* stream);
/* kin_ik_coll_batch (a static kin_sdf: scene_q / lds ignored) or kin_ik_coll_batch_scene (an attached one)
 * with a restart origin q_alt ([n_q(+3)][ldq], the layout of q; may alias q0 or q): attempt 0 starts
 * from q0; restart attempt 1 takes the free joint variables from q_alt instead of a seeded draw, and
 * every restart (1, 2, ...) takes its base columns from q_alt instead of q0; attempts >= 2 draw the
 * joints as before.  For the bistage solve (src/inverse_kinematics.jl:1-21): stage 2 starts from
 * stage 1's answer, whose base stage 1 has moved; with q_alt = the pose stage 1 started from, the
 * restarts leave that basin (PR2 fridge leg: DESIGN.md §4.6).  q_alt = NULL: exactly
 * kin_ik_coll_batch(_scene). */
KINHIP_API int kin_ik_coll_batch_alt(const kin_plan* p, const kin_sdf* sdf, const kin_ik_params* prm,
                                     const kin_ik_coll_params* cprm, const void* target, int64_t ldt,
                                     const void* scene_q, int64_t lds, const void* q0, const void* q_alt, void* q,
                                     int64_t ldq, int64_t n, int32_t* iters, void* err, int64_t lde, void* stream);

/* ------------------------------------------------------------------------- */
/* Planning constraints over waypoints (src/planning.jl) */
/* ------------------------------------------------------------------------- */
/* IneqConst (src/planning.jl:55-68) for N waypoints (configurations), any
 * number of trajectories side by side:
 *   vals [n_spheres][ldv]  min(dist, margin + 0.05) - margin
 *   jac  [n_spheres][n_q(+3)][ldj]  its gradient (0 where truncated), or NULL
 * i.e. the reference's val_vec[n_coll*(i-1) + s] and the diagonal block
 * jac_mat[n_dof*(i-1) + d, n_coll*(i-1) + s] of waypoint i. */
KINHIP_API int kin_ineq_const_batch(const kin_plan* coll_plan, const kin_sdf* sdf, double margin, const void* q,
                                    int64_t ldq, int64_t n, void* vals, int64_t ldv, void* jac, int64_t ldj,
                                    void* stream);
/* PoseConstraint (src/planning.jl:114-138) of one link for N configurations.
 * `p` must come from kin_plan_create with n_out = 1, jac_link = that link and
 * jac_flags = KIN_RPY_JAC | KIN_WITH_ROT (6 rows) or 0 (position only, 3 rows).
 *   target [12][ldt]  per-configuration target pose (3x4 column-major)
 *   poses  [12][ldp]  current pose (work + output, required)
 *   vals   [rows][ldv] [p - p*; rpy - rpy*]
 *   jac    [n_q(+3)][rows][ldj]  get_jacobian!(..., rpy_jac=true) (kin_plan_run layout; required) */
KINHIP_API int kin_pose_const_batch(const kin_plan* p, const void* target, int64_t ldt, const void* q, int64_t ldq,
                                    int64_t n, void* poses, int64_t ldp, void* vals, int64_t ldv, void* jac,
                                    int64_t ldj, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KINHIP_H */
