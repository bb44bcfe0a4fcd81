/*
 * kin_oracle.h -- CPU restatement of Kinematics.jl's hot path (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle and the timed CPU baseline ("port") for the
 * MI355X engine.  It is NOT part of the product: only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may load it, and only as the
 * checker.  The product path (libkinhip.so) never links or calls it.
 *
 * It restates, in reference-faithful form (per-config Mechanism state, cache
 * invalidation on every set, quaternion joint transforms, dense 4x4 fp64
 * products, explicit leaf->root stack, cached world joint axes):
 *   src/transform.jl:3-65, src/cache.jl:1-37, src/stack.jl:3-25,
 *   src/mechanism.jl:90-139, 199-277, src/algorithm.jl:1-131,
 *   src/inverse_kinematics.jl:38-50.
 * Third-party arithmetic restated (absent here): Rotations.jl 1.0.2
 * (UnitQuaternion normalisation, quaternion->RotMatrix, RotZYX extraction),
 * StaticArrays 1.0.1 (4x4 product).
 *
 * Pinned by: data/ground_truth.json (9 PR2 poses, with/without base) and the
 * reference's forward-difference Jacobian test (test/test_kinematics.jl:43-73),
 * see tests/test_oracle.py.
 *
 * Conventions: link/joint ids are 1-based like the reference; transforms are
 * 4x4 column-major (Julia SMatrix memory order).
 */
#ifndef KIN_ORACLE_H
#define KIN_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_FIXED = 0, OR_REVOLUTE = 1, OR_PRISMATIC = 2 };

typedef struct {
    int32_t n_links, n_joints;
    const int32_t* joint_type;  /* [n_joints] */
    const int32_t* joint_plink; /* [n_joints] 1-based */
    const int32_t* joint_clink; /* [n_joints] 1-based */
    const double* joint_pose;   /* [n_joints][16] column-major */
    const double* joint_axis;   /* [n_joints][3] */
    const double* joint_lower;  /* [n_joints] */
    const double* joint_upper;  /* [n_joints] */
    int32_t with_base;
} or_desc;

typedef struct or_mech or_mech;

or_mech* or_mech_create(const or_desc* d);
or_mech* or_mech_clone(const or_mech* m);
void or_mech_destroy(or_mech* m);
int32_t or_n_links(const or_mech* m);
int32_t or_n_joints(const or_mech* m);

/* src/mechanism.jl:223-231 -- angles has n (+3 if with_base) entries */
void or_set_joint_angles(or_mech* m, int32_t n, const int32_t* joint_ids, const double* angles);
/* src/mechanism.jl:199-200 */
void or_set_joint_angle(or_mech* m, int32_t joint_id, double angle);
/* src/mechanism.jl:203-214 */
void or_get_joint_angles(const or_mech* m, int32_t n, const int32_t* joint_ids, double* out);
void or_invalidate_cache(or_mech* m);
/* src/algorithm.jl:1-4 */
void or_get_transform(or_mech* m, int32_t link_id, double* out16);
/* src/algorithm.jl:83-106 (get_jacobian!: untouched entries stay as they are) */
int or_get_jacobian(or_mech* m, int32_t link_id, int32_t n, const int32_t* joint_ids,
                    int32_t with_rot, int32_t rpy_jac, double* mat_out /* rows x cols, col-major */);
/* src/mechanism.jl:277 */
int32_t or_is_relevant(const or_mech* m, int32_t joint_id, int32_t link_id);
/* src/mechanism.jl:238-267: adds a fixed child link; returns new link id */
int32_t or_add_new_link(or_mech* m, int32_t parent_link_id, const double* pose16);
/* src/transform.jl:45-48 -> [roll, pitch, yaw] */
void or_rpy(const double* tf16, double* out3);
/* src/algorithm.jl:116-131 (including the .+ sr_weight broadcast quirk) */
void or_point_ik_nakamura(or_mech* m, int32_t link_id, int32_t n, const int32_t* joint_ids,
                          const double* point3, double* angles_out);
/* src/inverse_kinematics.jl:38-50: returns sum(diff.^2); grad has n (+3) entries */
double or_ik_objective(or_mech* m, int32_t link_id, int32_t n, const int32_t* joint_ids,
                       const double* target16, int32_t with_rot, const double* angles, double* grad);

/* ---- batched drivers (one Mechanism per thread, the reference loop per config) ----
 * q: column c of the batch at q[c*ldq + i], c in [0, n_q (+3 if with_base)).
 * poses: [n_out][12][ldp]  (3x4 column-major per link: R11 R21 R31 R12 ... tx ty tz)
 * jac:   [n_cols][rows][ldj], rows = with_rot ? 6 : 3; n_cols = n_jac (+3 if with_base)
 * zero_fill=1 reproduces get_jacobian (zeros), 0 reproduces get_jacobian! on
 * whatever the caller's buffer holds. */
void or_fk_batch(const or_mech* proto, int64_t n, const double* q, int64_t ldq,
                 int32_t n_q, const int32_t* q_joint_ids, int32_t n_out, const int32_t* out_link_ids,
                 double* poses, int64_t ldp, int32_t n_threads);
void or_fk_jac_batch(const or_mech* proto, int64_t n, const double* q, int64_t ldq,
                     int32_t n_q, const int32_t* q_joint_ids, int32_t link_id,
                     int32_t n_jac, const int32_t* jac_joint_ids, int32_t with_rot, int32_t rpy_jac,
                     int32_t zero_fill, double* pose, int64_t ldp, double* jac, int64_t ldj,
                     int32_t n_threads);
/* Batched Nakamura point IK (config-independent starting angles q0 in q). */
void or_point_ik_nakamura_batch(const or_mech* proto, int64_t n, double* q, int64_t ldq,
                                int32_t n_q, const int32_t* q_joint_ids, int32_t link_id,
                                const double* points, int64_t ldpt, int32_t n_threads);

/* ---- build-defined damped-least-squares IK (config 4), restated for parity ----
 * Not a reference algorithm (the reference uses NLopt SLSQP, parity unpinned);
 * this is the CPU statement of the GPU kernel's algorithm so the kernel's
 * iterates can be checked.  See DESIGN.md "ik_dls".  Per iteration: e = [p* - p; log(R* R^T)],
 * dq = W J^T (J W J^T + lambda^2 I)^-1 e with W = diag(joint not held), |dq|_inf clamped to
 * max_step, q clamped to the limits; a joint is held in the next iteration when it sits on a limit
 * and J_k^T (...)^-1 e of this one pushes it further out (active set, one iteration behind). */
typedef struct {
    int32_t max_iters;
    double lambda;     /* damping */
    double tol_pos;    /* |dp| */
    double tol_rot;    /* |rotation error| (axis-angle) */
    double max_step;   /* clamp on |dq|_inf per iteration */
    int32_t with_rot;  /* 0: position only, 1: axis-angle residual, 2: the reference's [p* - p; rpy* - rpy]
                          residual (wrapped) with the rpy_jac Jacobian (src/inverse_kinematics.jl:38-50) */
    int32_t restarts;  /* attempts = restarts + 1, each max_iters / attempts iterations */
    uint64_t seed;     /* re-seed stream: ik_seed_u01(seed, config index, attempt, column) */
    double damp_err;   /* error-scaled damping: lambda^2 + damp_err * (|dp|^2 + |rot|^2) (0: fixed lambda) */
} or_ik_params;
/* the restart re-seed draw in [0, 1) shared by the oracle and the GPU kernel */
double or_ik_seed_u01(uint64_t seed, int64_t i, int32_t attempt, int32_t col);
/* log(Rt R^T) as a world rotation vector (the IK's rotation error); 4x4 column-major inputs */
void or_rot_error(const double* tgt16, const double* now16, double* w3);
void or_ik_dls_batch(const or_mech* proto, int64_t n, double* q, int64_t ldq, int32_t n_q,
                     const int32_t* q_joint_ids, int32_t link_id, const double* target, int64_t ldt,
                     const or_ik_params* prm, int32_t* iters_out, double* err_out, int32_t n_threads);

/* ---- signed distance fields and swept-sphere collision (src/sdf.jl, src/collision.jl) ----
 * Boxes: world pose (4x4 column-major) + full widths; the union is the min over
 * boxes (src/sdf.jl:108-114, argmin = first minimum). */
typedef struct {
    int32_t n_boxes;
    double* inv_pose;  /* [n][16] column-major inverse world poses (BoxSDF.inv_pose) */
    double* width;     /* [n][3] */
} or_union_sdf;
or_union_sdf* or_sdf_create(int32_t n_boxes, const double* poses16, const double* widths3);
void or_sdf_destroy(or_union_sdf* s);
/* BoxSDF value (src/sdf.jl:67-74) of box k at world point p */
double or_box_sdf(const or_union_sdf* s, int32_t k, const double* p);
/* UnionSDF value (src/sdf.jl:108-114); *argmin (0-based) may be NULL */
double or_union_sdf_value(const or_union_sdf* s, const double* p, int32_t* argmin);
/* gradient! of the union (src/sdf.jl:34-41, 116-119): forward difference, eps 1e-7, on the min box */
void or_union_sdf_gradient(const or_union_sdf* s, const double* p, double* grad3);
/* compute_coll_dists_and_grads! (src/collision.jl:67-94) for a batch: sphere k is link sph_links[k]
 * (its origin is the sphere centre, src/collision.jl:39-49) with radius radii[k].
 * dists: [n_sph][ldd]; grads (nullable): [n_sph][n_dof][ldg] with n_dof = n_q (+3 base);
 * dist > truncation -> value = truncation, gradient 0. */
void or_coll_batch(const or_mech* proto, const or_union_sdf* sdf, int64_t n, const double* q, int64_t ldq,
                   int32_t n_q, const int32_t* q_joint_ids, int32_t n_sph, const int32_t* sph_links,
                   const double* radii, double truncation, double* dists, int64_t ldd, double* grads,
                   int64_t ldg, int32_t n_threads);

/* build-defined collision-aware IK (kin_ik_coll_batch), restated: see kin_oracle.c.
 * cprm = {margin, band, weight, feas}; err_out [3][n]: |dp|, |rot|, min sphere distance.
 * q_alt (nullable, [n_q(+3)][ldq]): restart attempt 1 starts the relevant joints from it instead of a draw,
 * and every restart the base (kin_ik_coll_batch_alt). */
void or_ik_coll_batch(const or_mech* proto, const or_union_sdf* sdf, int64_t n, double* q, int64_t ldq, int32_t n_q,
                      const int32_t* qids, int32_t link_id, const double* target, int64_t ldt, const or_ik_params* prm,
                      const double* cprm, int32_t n_sph, const int32_t* sph, const double* radii,
                      const or_union_sdf* const* sdfs, const double* q_alt, int32_t* iters_out, double* err_out,
                      int32_t n_threads);

#ifdef __cplusplus
}
#endif
#endif
