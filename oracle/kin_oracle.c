/*
 * kin_oracle.c -- CPU restatement of Kinematics.jl's FK / Jacobian / IK hot
 * path.  TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline); the
 * product library never links this file.  See kin_oracle.h for the header
 * contract and the reference files restated.
 *
 * Structure deliberately mirrors the reference (it is the "reference-faithful"
 * CPU baseline of BASELINE.md): a Mechanism with tf/axis caches that are
 * invalidated on every angle set, a PseudoStack walk from the leaf to the
 * shallowest cached ancestor, quaternion joint rotations and dense 4x4
 * products.
 */
#include "kin_oracle.h"


#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* Transform (src/transform.jl): 4x4 column-major, index (i,j) -> i+4j  */
/* ------------------------------------------------------------------ */
typedef struct { double m[16]; } tf_t;
#define M(t, i, j) ((t).m[(i) + 4 * (j)])

static tf_t tf_identity(void) {  /* zero(Transform) == one(Transform): src/transform.jl:50-56 */
    tf_t t; memset(&t, 0, sizeof t);
    t.m[0] = t.m[5] = t.m[10] = t.m[15] = 1.0;
    return t;
}

/* dense 4x4 product, src/transform.jl:58-60 (StaticArrays unrolled mul) */
static tf_t tf_mul(const tf_t* a, const tf_t* b) {
    tf_t c;
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) {
            double s = M(*a, i, 0) * M(*b, 0, j);
            s += M(*a, i, 1) * M(*b, 1, j);
            s += M(*a, i, 2) * M(*b, 2, j);
            s += M(*a, i, 3) * M(*b, 3, j);
            M(c, i, j) = s;
        }
    return c;
}

/* Rotations.jl 1.0.2: UnitQuaternion(w,x,y,z) normalises, RotMatrix(q). */
static void quat_to_rot(double w, double x, double y, double z, double R[9] /* col-major 3x3 */) {
    double n = sqrt(w * w + x * x + y * y + z * z);
    w /= n; x /= n; y /= n; z /= n;
    double ww = w * w, xx = x * x, yy = y * y, zz = z * z;
    double xy = x * y, zw = w * z, xz = x * z, yw = y * w, yz = y * z, xw = w * x;
    R[0] = ww + xx - yy - zz; R[3] = 2 * (xy - zw);      R[6] = 2 * (xz + yw);
    R[1] = 2 * (xy + zw);     R[4] = ww - xx + yy - zz;  R[7] = 2 * (yz - xw);
    R[2] = 2 * (xz - yw);     R[5] = 2 * (yz + xw);      R[8] = ww - xx - yy + zz;
}

/* Transform(trans, rot) / Transform(rot): src/transform.jl:7-23 */
static tf_t tf_from_rot_trans(const double R[9], double tx, double ty, double tz) {
    tf_t t = tf_identity();
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) M(t, i, j) = R[i + 3 * j];
    M(t, 0, 3) = tx; M(t, 1, 3) = ty; M(t, 2, 3) = tz;
    return t;
}

/* base_pose_to_transform: src/transform.jl:33-37 */
static tf_t base_pose_to_transform(const double p[3]) {
    double R[9];
    quat_to_rot(cos(0.5 * p[2]), 0.0, 0.0, sin(0.5 * p[2]), R);
    return tf_from_rot_trans(R, p[0], p[1], 0.0);
}

/* RotZYX(rotation(t)) -> [theta3, theta2, theta1] = [roll, pitch, yaw]: src/transform.jl:45-48 */
static void rpy_of(const tf_t* t, double out[3]) {
    double r11 = M(*t, 0, 0), r21 = M(*t, 1, 0), r31 = M(*t, 2, 0);
    double r12 = M(*t, 0, 1), r22 = M(*t, 1, 1);
    double r13 = M(*t, 0, 2), r23 = M(*t, 1, 2);
    double t1 = atan2(r21, r11);
    double ct1 = cos(t1), st1 = sin(t1);
    double t2 = atan2(-r31, r21 * st1 + r11 * ct1);
    double t3 = atan2(r13 * st1 - r23 * ct1, r22 * ct1 - r12 * st1);
    out[0] = t3; out[1] = t2; out[2] = t1;
}

void or_rpy(const double* tf16, double* out3) {
    tf_t t; memcpy(t.m, tf16, sizeof t.m);
    rpy_of(&t, out3);
}

/* ------------------------------------------------------------------ */
/* Mechanism (src/mechanism.jl)                                         */
/* ------------------------------------------------------------------ */
typedef struct { double origin[3], axis[3]; } faxis_t; /* FloatingAxis :105-115 */

struct or_mech {
    int32_t n_links, n_joints, cap_links, cap_joints;
    /* links */
    int32_t* plink;   /* 1-based, -1 root */
    int32_t* pjoint;  /* 1-based, -1 root */
    int32_t* nchild;
    int32_t** clinks; /* children, in joint order (load_urdf.jl:69-71) */
    int32_t* ccap;
    /* joints */
    int32_t* jtype;
    int32_t* jplink;
    int32_t* jclink;
    tf_t* jpose;
    double (*jaxis)[3];
    double* jlower;
    double* jupper;
    /* state */
    double* angles;
    double base_pose[3];
    int32_t with_base;
    tf_t* tf_cache; uint8_t* tf_valid;      /* CacheVector{Transform} */
    faxis_t* ax_cache; uint8_t* ax_valid;   /* CacheVector{FloatingAxis} */
    uint8_t* rptable;                        /* [joint][link], create_rptable :117-139 */
    tf_t* tf_stack; int32_t* id_stack; int32_t top; /* PseudoStack :3-25 */
};

static void* xrealloc(void* p, size_t n) { void* q = realloc(p, n ? n : 1); if (!q) abort(); return q; }

static void push_child(or_mech* m, int32_t l /*0-based*/, int32_t c /*1-based*/) {
    if (m->nchild[l] == m->ccap[l]) {
        m->ccap[l] = m->ccap[l] ? 2 * m->ccap[l] : 4;
        m->clinks[l] = (int32_t*)xrealloc(m->clinks[l], sizeof(int32_t) * m->ccap[l]);
    }
    m->clinks[l][m->nchild[l]++] = c;
}

static void rp_mark(or_mech* m, int32_t j, int32_t l /*1-based*/) {
    m->rptable[(size_t)j * m->n_links + (l - 1)] = 1;
    for (int32_t k = 0; k < m->nchild[l - 1]; ++k) rp_mark(m, j, m->clinks[l - 1][k]);
}

static void build_rptable(or_mech* m) {
    free(m->rptable);
    m->rptable = (uint8_t*)calloc((size_t)m->n_joints * m->n_links + 1, 1);
    for (int32_t j = 0; j < m->n_joints; ++j) rp_mark(m, j, m->jclink[j]);
}

static void alloc_state(or_mech* m) {
    m->tf_cache = (tf_t*)xrealloc(m->tf_cache, sizeof(tf_t) * m->n_links);
    m->tf_valid = (uint8_t*)xrealloc(m->tf_valid, m->n_links);
    m->ax_cache = (faxis_t*)xrealloc(m->ax_cache, sizeof(faxis_t) * m->n_joints);
    m->ax_valid = (uint8_t*)xrealloc(m->ax_valid, m->n_joints);
    m->tf_stack = (tf_t*)xrealloc(m->tf_stack, sizeof(tf_t) * m->n_links);
    m->id_stack = (int32_t*)xrealloc(m->id_stack, sizeof(int32_t) * m->n_links);
    memset(m->tf_valid, 0, m->n_links);
    memset(m->ax_valid, 0, m->n_joints);
    m->top = 0;
}

or_mech* or_mech_create(const or_desc* d) {
    or_mech* m = (or_mech*)calloc(1, sizeof(or_mech));
    m->n_links = d->n_links; m->n_joints = d->n_joints;
    int32_t L = d->n_links, J = d->n_joints;
    m->plink = (int32_t*)malloc(sizeof(int32_t) * (L + 1));
    m->pjoint = (int32_t*)malloc(sizeof(int32_t) * (L + 1));
    m->nchild = (int32_t*)calloc(L + 1, sizeof(int32_t));
    m->ccap = (int32_t*)calloc(L + 1, sizeof(int32_t));
    m->clinks = (int32_t**)calloc(L + 1, sizeof(int32_t*));
    for (int32_t l = 0; l < L; ++l) { m->plink[l] = -1; m->pjoint[l] = -1; }
    m->jtype = (int32_t*)malloc(sizeof(int32_t) * (J + 1));
    m->jplink = (int32_t*)malloc(sizeof(int32_t) * (J + 1));
    m->jclink = (int32_t*)malloc(sizeof(int32_t) * (J + 1));
    m->jpose = (tf_t*)malloc(sizeof(tf_t) * (J + 1));
    m->jaxis = (double (*)[3])malloc(sizeof(double[3]) * (J + 1));
    m->jlower = (double*)malloc(sizeof(double) * (J + 1));
    m->jupper = (double*)malloc(sizeof(double) * (J + 1));
    m->angles = (double*)calloc(J + 1, sizeof(double));
    for (int32_t j = 0; j < J; ++j) {
        m->jtype[j] = d->joint_type[j];
        m->jplink[j] = d->joint_plink[j];
        m->jclink[j] = d->joint_clink[j];
        memcpy(m->jpose[j].m, d->joint_pose + 16 * j, sizeof(double) * 16);
        memcpy(m->jaxis[j], d->joint_axis + 3 * j, sizeof(double) * 3);
        m->jlower[j] = d->joint_lower ? d->joint_lower[j] : -INFINITY;
        m->jupper[j] = d->joint_upper ? d->joint_upper[j] : INFINITY;
        /* parse_urdf tree wiring, src/load_urdf.jl:69-75 */
        push_child(m, m->jplink[j] - 1, m->jclink[j]);
        m->plink[m->jclink[j] - 1] = m->jplink[j];
        m->pjoint[m->jclink[j] - 1] = j + 1;
    }
    m->with_base = d->with_base;
    m->cap_links = L + 1; m->cap_joints = J + 1;
    alloc_state(m);
    build_rptable(m);
    return m;
}

or_mech* or_mech_clone(const or_mech* s) {
    or_desc d;
    int32_t J = s->n_joints;
    double* pose = (double*)malloc(sizeof(double) * 16 * (J + 1));
    double* axis = (double*)malloc(sizeof(double) * 3 * (J + 1));
    for (int32_t j = 0; j < J; ++j) {
        memcpy(pose + 16 * j, s->jpose[j].m, sizeof(double) * 16);
        memcpy(axis + 3 * j, s->jaxis[j], sizeof(double) * 3);
    }
    d.n_links = s->n_links; d.n_joints = J;
    d.joint_type = s->jtype; d.joint_plink = s->jplink; d.joint_clink = s->jclink;
    d.joint_pose = pose; d.joint_axis = axis; d.joint_lower = s->jlower; d.joint_upper = s->jupper;
    d.with_base = s->with_base;
    or_mech* m = or_mech_create(&d);
    memcpy(m->angles, s->angles, sizeof(double) * J);
    memcpy(m->base_pose, s->base_pose, sizeof m->base_pose);
    free(pose); free(axis);
    return m;
}

void or_mech_destroy(or_mech* m) {
    if (!m) return;
    for (int32_t l = 0; l < m->n_links; ++l) free(m->clinks[l]);
    free(m->clinks); free(m->plink); free(m->pjoint); free(m->nchild); free(m->ccap);
    free(m->jtype); free(m->jplink); free(m->jclink); free(m->jpose); free(m->jaxis);
    free(m->jlower); free(m->jupper); free(m->angles);
    free(m->tf_cache); free(m->tf_valid); free(m->ax_cache); free(m->ax_valid);
    free(m->rptable); free(m->tf_stack); free(m->id_stack);
    free(m);
}

int32_t or_n_links(const or_mech* m) { return m->n_links; }
int32_t or_n_joints(const or_mech* m) { return m->n_joints; }

/* invalidate_cache!: src/mechanism.jl:270 */
void or_invalidate_cache(or_mech* m) {
    memset(m->tf_valid, 0, m->n_links);
    memset(m->ax_valid, 0, m->n_joints);
}

void or_set_joint_angle(or_mech* m, int32_t joint_id, double angle) {
    m->angles[joint_id - 1] = angle;
    or_invalidate_cache(m);
}

void or_set_joint_angles(or_mech* m, int32_t n, const int32_t* ids, const double* angles) {
    for (int32_t i = 0; i < n; ++i) m->angles[ids[i] - 1] = angles[i];
    if (m->with_base)
        for (int k = 0; k < 3; ++k) m->base_pose[k] = angles[n + k];
    or_invalidate_cache(m);
}

void or_get_joint_angles(const or_mech* m, int32_t n, const int32_t* ids, double* out) {
    for (int32_t i = 0; i < n; ++i) out[i] = m->angles[ids[i] - 1];
    if (m->with_base)
        for (int k = 0; k < 3; ++k) out[n + k] = m->base_pose[k];
}

int32_t or_is_relevant(const or_mech* m, int32_t joint_id, int32_t link_id) {
    return m->rptable[(size_t)(joint_id - 1) * m->n_links + (link_id - 1)];
}

/* joint_transform: src/mechanism.jl:90-103 */
static tf_t joint_transform(const or_mech* m, int32_t j /*0-based*/, double angle) {
    switch (m->jtype[j]) {
    case OR_FIXED:
        return m->jpose[j];
    case OR_REVOLUTE: {
        if (angle == 0.0) return m->jpose[j];
        double s = sin(0.5 * angle), c = cos(0.5 * angle);
        double R[9];
        quat_to_rot(c, m->jaxis[j][0] * s, m->jaxis[j][1] * s, m->jaxis[j][2] * s, R);
        tf_t r = tf_from_rot_trans(R, 0.0, 0.0, 0.0);
        return tf_mul(&m->jpose[j], &r);
    }
    default: { /* prismatic */
        if (angle == 0.0) return m->jpose[j];
        tf_t tr = tf_identity();
        M(tr, 0, 3) = m->jaxis[j][0] * angle;
        M(tr, 1, 3) = m->jaxis[j][1] * angle;
        M(tr, 2, 3) = m->jaxis[j][2] * angle;
        return tf_mul(&m->jpose[j], &tr);
    }
    }
}

/* _get_shallowest_cache!: src/algorithm.jl:23-37 */
static tf_t shallowest_cache(or_mech* m, int32_t hlink /*1-based*/) {
    while (m->plink[hlink - 1] != -1) {
        if (m->tf_valid[hlink - 1]) return m->tf_cache[hlink - 1];
        int32_t hj = m->pjoint[hlink - 1] - 1;
        tf_t tf_local = joint_transform(m, hj, m->angles[hj]);
        m->tf_stack[m->top] = tf_local;
        m->id_stack[m->top] = hlink;
        m->top++;
        hlink = m->plink[hlink - 1];
    }
    return m->with_base ? base_pose_to_transform(m->base_pose) : tf_identity();
}

/* get_transform / _get_transform: src/algorithm.jl:1-21 */
static tf_t get_transform(or_mech* m, int32_t link_id) {
    if (m->tf_valid[link_id - 1]) return m->tf_cache[link_id - 1];
    tf_t w = shallowest_cache(m, link_id);
    while (m->top > 0) {
        m->top--;
        int32_t hid = m->id_stack[m->top];
        w = tf_mul(&w, &m->tf_stack[m->top]);
        m->tf_cache[hid - 1] = w;
        m->tf_valid[hid - 1] = 1;
    }
    return w;
}

void or_get_transform(or_mech* m, int32_t link_id, double* out16) {
    tf_t t = get_transform(m, link_id);
    memcpy(out16, t.m, sizeof t.m);
}

/* _get_joint_axis: src/algorithm.jl:42-54 */
static faxis_t joint_axis(or_mech* m, int32_t j /*0-based*/) {
    if (m->ax_valid[j]) return m->ax_cache[j];
    tf_t tp = get_transform(m, m->jplink[j]);
    tf_t th = tf_mul(&tp, &m->jpose[j]);
    faxis_t f;
    for (int i = 0; i < 3; ++i) {
        f.origin[i] = M(th, i, 3);
        f.axis[i] = M(th, i, 0) * m->jaxis[j][0] + M(th, i, 1) * m->jaxis[j][1] + M(th, i, 2) * m->jaxis[j][2];
    }
    m->ax_cache[j] = f;
    m->ax_valid[j] = 1;
    return f;
}

/* rpy_derivative!: src/algorithm.jl:56-63 */
static void rpy_derivative(const double rpy[3], const double ax[3], double out[3]) {
    double a2 = -rpy[1], a3 = -rpy[2];
    double x = ax[0], y = ax[1], z = ax[2];
    out[0] = cos(a3) / cos(a2) * x - sin(a3) / cos(a2) * y;
    out[1] = sin(a3) * x + cos(a3) * y;
    out[2] = -cos(a3) * sin(a2) / cos(a2) * x + sin(a3) * sin(a2) / cos(a2) * y + z;
}

/* get_jacobian!: src/algorithm.jl:83-106.  Returns -3 (MethodError) for a
 * relevant fixed joint, which has no joint_jacobian! method. */
int or_get_jacobian(or_mech* m, int32_t link_id, int32_t n, const int32_t* ids,
                    int32_t with_rot, int32_t rpy_jac, double* J) {
    int rows = with_rot ? 6 : 3;
    tf_t tl = get_transform(m, link_id);
    double p[3] = {M(tl, 0, 3), M(tl, 1, 3), M(tl, 2, 3)};
    double rpy[3];
    int have_rpy = 0;
    for (int32_t i = 0; i < n; ++i) {
        int32_t j = ids[i] - 1;
        if (!or_is_relevant(m, ids[i], link_id)) continue;
        double* col = J + (size_t)rows * i;
        if (m->jtype[j] == OR_FIXED) return -3;
        faxis_t f = joint_axis(m, j);
        if (m->jtype[j] == OR_REVOLUTE) {
            double d[3] = {p[0] - f.origin[0], p[1] - f.origin[1], p[2] - f.origin[2]};
            col[0] = f.axis[1] * d[2] - f.axis[2] * d[1];
            col[1] = f.axis[2] * d[0] - f.axis[0] * d[2];
            col[2] = f.axis[0] * d[1] - f.axis[1] * d[0];
            if (with_rot) {
                if (rpy_jac) {
                    if (!have_rpy) { rpy_of(&tl, rpy); have_rpy = 1; }
                    rpy_derivative(rpy, f.axis, col + 3);
                } else {
                    col[3] = f.axis[0]; col[4] = f.axis[1]; col[5] = f.axis[2];
                }
            }
        } else { /* prismatic: rows 4:6 untouched */
            col[0] = f.axis[0]; col[1] = f.axis[1]; col[2] = f.axis[2];
        }
    }
    if (m->with_base) {
        double x = p[0] - m->base_pose[0], y = p[1] - m->base_pose[1];
        double* c1 = J + (size_t)rows * n;
        double* c2 = c1 + rows;
        double* c3 = c2 + rows;
        c1[0] = 1; c1[1] = 0; c1[2] = 0;
        c2[0] = 0; c2[1] = 1; c2[2] = 0;
        c3[0] = -y; c3[1] = x; c3[2] = 0;
        if (with_rot) {
            c1[3] = c1[4] = c1[5] = 0;
            c2[3] = c2[4] = c2[5] = 0;
            c3[3] = 0; c3[4] = 0; c3[5] = 1.0;
        }
    }
    return 0;
}

/* add_new_link: src/mechanism.jl:238-267 */
int32_t or_add_new_link(or_mech* m, int32_t parent, const double* pose16) {
    int32_t L = m->n_links, J = m->n_joints;
    m->plink = (int32_t*)xrealloc(m->plink, sizeof(int32_t) * (L + 1));
    m->pjoint = (int32_t*)xrealloc(m->pjoint, sizeof(int32_t) * (L + 1));
    m->nchild = (int32_t*)xrealloc(m->nchild, sizeof(int32_t) * (L + 1));
    m->ccap = (int32_t*)xrealloc(m->ccap, sizeof(int32_t) * (L + 1));
    m->clinks = (int32_t**)xrealloc(m->clinks, sizeof(int32_t*) * (L + 1));
    m->jtype = (int32_t*)xrealloc(m->jtype, sizeof(int32_t) * (J + 1));
    m->jplink = (int32_t*)xrealloc(m->jplink, sizeof(int32_t) * (J + 1));
    m->jclink = (int32_t*)xrealloc(m->jclink, sizeof(int32_t) * (J + 1));
    m->jpose = (tf_t*)xrealloc(m->jpose, sizeof(tf_t) * (J + 1));
    m->jaxis = (double (*)[3])xrealloc(m->jaxis, sizeof(double[3]) * (J + 1));
    m->jlower = (double*)xrealloc(m->jlower, sizeof(double) * (J + 1));
    m->jupper = (double*)xrealloc(m->jupper, sizeof(double) * (J + 1));
    m->angles = (double*)xrealloc(m->angles, sizeof(double) * (J + 1));
    m->plink[L] = parent; m->pjoint[L] = J + 1; m->nchild[L] = 0; m->ccap[L] = 0; m->clinks[L] = NULL;
    push_child(m, parent - 1, L + 1);
    m->jtype[J] = OR_FIXED; m->jplink[J] = parent; m->jclink[J] = L + 1;
    memcpy(m->jpose[J].m, pose16, sizeof(double) * 16);
    m->jaxis[J][0] = 1; m->jaxis[J][1] = 0; m->jaxis[J][2] = 0;
    m->jlower[J] = -INFINITY; m->jupper[J] = INFINITY;
    m->angles[J] = 0.0;
    m->n_links = L + 1; m->n_joints = J + 1;
    alloc_state(m);
    build_rptable(m);
    return L + 1;
}

/* ---- small dense helpers ---- */
static void inv3(const double A[9] /*col-major*/, double B[9]) {
    double a = A[0], b = A[3], c = A[6], d = A[1], e = A[4], f = A[7], g = A[2], h = A[5], i = A[8];
    double A_ = e * i - f * h, B_ = -(d * i - f * g), C_ = d * h - e * g;
    double det = a * A_ + b * B_ + c * C_;
    B[0] = A_ / det; B[3] = -(b * i - c * h) / det; B[6] = (b * f - c * e) / det;
    B[1] = B_ / det; B[4] = (a * i - c * g) / det;  B[7] = -(a * f - c * d) / det;
    B[2] = C_ / det; B[5] = -(a * h - b * g) / det; B[8] = (a * e - b * d) / det;
}

/* point_inverse_kinematics_nakamura: src/algorithm.jl:116-131 */
void or_point_ik_nakamura(or_mech* m, int32_t link_id, int32_t n, const int32_t* ids,
                          const double* pd, double* angles) {
    double* jac = (double*)malloc(sizeof(double) * 3 * (n + 3));
    or_get_joint_angles(m, n, ids, angles);
    int32_t ndof = n; /* SizedVector{n_dof}: base columns are not part of it */
    for (int it = 0; it < 50; ++it) {
        /* set_joint_angles(m, joints, angles) with angles of length n */
        for (int32_t i = 0; i < n; ++i) m->angles[ids[i] - 1] = angles[i];
        or_invalidate_cache(m);
        tf_t t = get_transform(m, link_id);
        double pn[3] = {M(t, 0, 3), M(t, 1, 3), M(t, 2, 3)};
        memset(jac, 0, sizeof(double) * 3 * (n + 3));
        int32_t wb = m->with_base; m->with_base = 0;  /* 3 x n_dof buffer */
        or_get_jacobian(m, link_id, n, ids, 0, 0, jac);
        m->with_base = wb;
        double JJ[9];
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 3; ++r) {
                double s = 0;
                for (int32_t k = 0; k < ndof; ++k) s += jac[r + 3 * k] * jac[c + 3 * k];
                JJ[r + 3 * c] = s + 1.0; /* `.+ sr_weight`: broadcast onto EVERY entry (quirk) */
            }
        double Ji[9];
        inv3(JJ, Ji);
        double dp[3] = {pd[0] - pn[0], pd[1] - pn[1], pd[2] - pn[2]};
        double y[3];
        for (int r = 0; r < 3; ++r) y[r] = Ji[r] * dp[0] + Ji[r + 3] * dp[1] + Ji[r + 6] * dp[2];
        for (int32_t k = 0; k < ndof; ++k)
            angles[k] += jac[3 * k] * y[0] + jac[3 * k + 1] * y[1] + jac[3 * k + 2] * y[2];
    }
    free(jac);
}

/* f_objective: src/inverse_kinematics.jl:38-50 */
double or_ik_objective(or_mech* m, int32_t link_id, int32_t n, const int32_t* ids,
                       const double* target16, int32_t with_rot, const double* angles, double* grad) {
    int32_t ndof = n + (m->with_base ? 3 : 0);
    int rows = with_rot ? 6 : 3;
    or_set_joint_angles(m, n, ids, angles);
    tf_t now = get_transform(m, link_id);
    tf_t tgt; memcpy(tgt.m, target16, sizeof tgt.m);
    double diff[6];
    for (int i = 0; i < 3; ++i) diff[i] = M(tgt, i, 3) - M(now, i, 3);
    if (with_rot) {
        double r0[3], r1[3];
        rpy_of(&tgt, r0); rpy_of(&now, r1);
        for (int i = 0; i < 3; ++i) diff[3 + i] = r0[i] - r1[i];
    }
    double* jac = (double*)calloc((size_t)rows * ndof, sizeof(double));
    or_get_jacobian(m, link_id, n, ids, with_rot, 1, jac);
    double f = 0;
    for (int r = 0; r < rows; ++r) f += diff[r] * diff[r];
    if (grad)
        for (int32_t k = 0; k < ndof; ++k) {
            double s = 0;
            for (int r = 0; r < rows; ++r) s += jac[r + rows * k] * diff[r];
            grad[k] = -2 * s;
        }
    free(jac);
    return f;
}

/* ------------------------------------------------------------------ */
/* Batched drivers                                                      */
/* ------------------------------------------------------------------ */
static int nthreads_of(int32_t t) {
#ifdef _OPENMP
    return t > 0 ? t : omp_get_max_threads();
#else
    (void)t; return 1;
#endif
}

void or_fk_batch(const or_mech* proto, int64_t n, const double* q, int64_t ldq,
                 int32_t n_q, const int32_t* qids, int32_t n_out, const int32_t* out_ids,
                 double* poses, int64_t ldp, int32_t n_threads) {
    int nt = nthreads_of(n_threads);
    int32_t ncolq = n_q + (proto->with_base ? 3 : 0);
#pragma omp parallel num_threads(nt)
    {
        or_mech* m = or_mech_clone(proto);
        double* a = (double*)malloc(sizeof(double) * (ncolq + 1));
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            for (int32_t c = 0; c < ncolq; ++c) a[c] = q[c * ldq + i];
            or_set_joint_angles(m, n_q, qids, a);
            for (int32_t o = 0; o < n_out; ++o) {
                tf_t t = get_transform(m, out_ids[o]);
                double* dst = poses + (size_t)o * 12 * ldp + i;
                for (int k = 0; k < 12; ++k) dst[(size_t)k * ldp] = t.m[(k / 3) * 4 + (k % 3)];
            }
        }
        free(a);
        or_mech_destroy(m);
    }
}

void or_fk_jac_batch(const or_mech* proto, int64_t n, const double* q, int64_t ldq,
                     int32_t n_q, const int32_t* qids, int32_t link_id,
                     int32_t n_jac, const int32_t* jids, int32_t with_rot, int32_t rpy_jac,
                     int32_t zero_fill, double* pose, int64_t ldp, double* jac, int64_t ldj,
                     int32_t n_threads) {
    int nt = nthreads_of(n_threads);
    int32_t ncolq = n_q + (proto->with_base ? 3 : 0);
    int32_t ncolj = n_jac + (proto->with_base ? 3 : 0);
    int rows = with_rot ? 6 : 3;
#pragma omp parallel num_threads(nt)
    {
        or_mech* m = or_mech_clone(proto);
        double* a = (double*)malloc(sizeof(double) * (ncolq + 1));
        double* J = (double*)malloc(sizeof(double) * rows * (ncolj + 1));
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            for (int32_t c = 0; c < ncolq; ++c) a[c] = q[c * ldq + i];
            or_set_joint_angles(m, n_q, qids, a);
            if (pose) {
                tf_t t = get_transform(m, link_id);
                for (int k = 0; k < 12; ++k) pose[(size_t)k * ldp + i] = t.m[(k / 3) * 4 + (k % 3)];
            }
            if (jac) {
                for (int32_t c = 0; c < ncolj; ++c)
                    for (int r = 0; r < rows; ++r)
                        J[r + rows * c] = zero_fill ? 0.0 : jac[((size_t)c * rows + r) * ldj + i];
                or_get_jacobian(m, link_id, n_jac, jids, with_rot, rpy_jac, J);
                for (int32_t c = 0; c < ncolj; ++c)
                    for (int r = 0; r < rows; ++r) jac[((size_t)c * rows + r) * ldj + i] = J[r + rows * c];
            }
        }
        free(a); free(J);
        or_mech_destroy(m);
    }
}

void or_point_ik_nakamura_batch(const or_mech* proto, int64_t n, double* q, int64_t ldq,
                                int32_t n_q, const int32_t* qids, int32_t link_id,
                                const double* pts, int64_t ldpt, int32_t n_threads) {
    int nt = nthreads_of(n_threads);
#pragma omp parallel num_threads(nt)
    {
        or_mech* m = or_mech_clone(proto);
        double* a = (double*)malloc(sizeof(double) * (n_q + 3));
        double* out = (double*)malloc(sizeof(double) * (n_q + 3));
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            for (int32_t c = 0; c < n_q; ++c) m->angles[qids[c] - 1] = q[c * ldq + i];
            or_invalidate_cache(m);
            double p[3] = {pts[i], pts[ldpt + i], pts[2 * ldpt + i]};
            or_point_ik_nakamura(m, link_id, n_q, qids, p, out);
            for (int32_t c = 0; c < n_q; ++c) q[c * ldq + i] = out[c];
        }
        free(a); free(out);
        or_mech_destroy(m);
    }
}

/* ---- build-defined DLS IK (see header) ---- */
static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double or_ik_seed_u01(uint64_t seed, int64_t i, int32_t attempt, int32_t col) {
    const uint64_t key = (uint64_t)i * 131ull + (uint64_t)attempt * 31ull + (uint64_t)col + 1ull;
    return (double)(splitmix64(seed + 0x9E3779B97F4A7C15ull * key) >> 11) * (1.0 / 9007199254740992.0);
}

/* world-frame rotation vector w with exp([w]) * R = Rt, i.e. log(Rt * R^T) */
static void rot_error(const tf_t* tgt, const tf_t* now, double w[3]) {
    double E[9]; /* col-major E = Rt * R^T */
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i)
            E[i + 3 * j] = M(*tgt, i, 0) * M(*now, j, 0) + M(*tgt, i, 1) * M(*now, j, 1) + M(*tgt, i, 2) * M(*now, j, 2);
    double v0 = 0.5 * (E[2 + 3 * 1] - E[1 + 3 * 2]);
    double v1 = 0.5 * (E[0 + 3 * 2] - E[2 + 3 * 0]);
    double v2 = 0.5 * (E[1 + 3 * 0] - E[0 + 3 * 1]);
    double s = sqrt(v0 * v0 + v1 * v1 + v2 * v2);
    double c = 0.5 * (E[0] + E[4] + E[8] - 1.0);
    double th = atan2(s, c);
    if (s > 1e-7) {
        double k = th / s;
        w[0] = v0 * k; w[1] = v1 * k; w[2] = v2 * k;
    } else if (c > 0) {
        w[0] = v0; w[1] = v1; w[2] = v2;
    } else { /* angle ~ pi: axis from the symmetric part */
        int b = 0;
        if (E[4] > E[b * 4]) b = 1;
        if (E[8] > E[b * 4]) b = 2;
        double a[3];
        for (int i = 0; i < 3; ++i) a[i] = 0.25 * (E[i + 3 * b] + E[b + 3 * i]); /* u_i u_b (E = 2uu^T - I) */
        a[b] = 0.5 * (E[b * 4] + 1.0);                                            /* u_b^2 */
        double nn = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        for (int i = 0; i < 3; ++i) w[i] = a[i] / nn * th;
    }
}

/* exported for the known-answer test of the angle ~ pi branch (tests/test_oracle.py) */
void or_rot_error(const double* tgt16, const double* now16, double* w3) {
    tf_t a, b;
    memcpy(a.m, tgt16, sizeof a.m);
    memcpy(b.m, now16, sizeof b.m);
    rot_error(&a, &b, w3);
}

/* Cholesky solve of symmetric positive definite A (n x n, col-major, n <= 64), in place on b.  Each pivot's
 * reciprocal 1 / sqrt(d) is formed once and multiplies (the kernels' fp64 form: k_ik_dls, k_ik_tree). */
static void chol_solve(double* A, int n, double* b) {
    double ip[64];
    for (int j = 0; j < n; ++j) {
        double d = A[j + n * j];
        for (int k = 0; k < j; ++k) d -= A[j + n * k] * A[j + n * k];
        d = sqrt(d);
        A[j + n * j] = d;
        ip[j] = 1.0 / d;
        for (int i = j + 1; i < n; ++i) {
            double s = A[i + n * j];
            for (int k = 0; k < j; ++k) s -= A[i + n * k] * A[j + n * k];
            A[i + n * j] = s * ip[j];
        }
    }
    for (int i = 0; i < n; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= A[i + n * k] * b[k];
        b[i] = s * ip[i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = b[i];
        for (int k = i + 1; k < n; ++k) s -= A[k + n * i] * b[k];
        b[i] = s * ip[i];
    }
}

void or_ik_dls_batch(const or_mech* proto, int64_t n, double* q, int64_t ldq, int32_t n_q,
                     const int32_t* qids, int32_t link_id, const double* target, int64_t ldt,
                     const or_ik_params* prm, int32_t* iters_out, double* err_out, int32_t n_threads) {
    int nt = nthreads_of(n_threads);
    int32_t ndof = n_q + (proto->with_base ? 3 : 0);
    int rows = prm->with_rot ? 6 : 3;
#pragma omp parallel num_threads(nt)
    {
        or_mech* m = or_mech_clone(proto);
        double* a = (double*)malloc(sizeof(double) * (ndof + 1));
        double* J = (double*)malloc(sizeof(double) * 6 * (ndof + 1));
        double* Jw = (double*)malloc(sizeof(double) * 6 * (ndof + 1));
        double* lo = (double*)malloc(sizeof(double) * (ndof + 1));
        double* hi = (double*)malloc(sizeof(double) * (ndof + 1));
        for (int32_t c = 0; c < ndof; ++c) { /* joints that cannot move the link are left untouched */
            int rel = c < n_q && or_is_relevant(m, qids[c], link_id);
            lo[c] = rel ? m->jlower[qids[c] - 1] : -INFINITY;
            hi[c] = rel ? m->jupper[qids[c] - 1] : INFINITY;
        }
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            tf_t tgt = tf_identity();
            for (int k = 0; k < 12; ++k) tgt.m[(k / 3) * 4 + (k % 3)] = target[(size_t)k * ldt + i];
            for (int32_t c = 0; c < ndof; ++c) a[c] = q[c * ldq + i];
            int32_t it = 0;
            double ep = 0, er = 0;
            const int32_t attempt_len = prm->restarts > 0 ? prm->max_iters / (prm->restarts + 1) : 0;
            double a0[64];
            int held[64];
            for (int32_t c = 0; c < ndof; ++c) { a0[c] = a[c]; held[c] = 0; }
            for (;; ++it) {
                or_set_joint_angles(m, n_q, qids, a);
                tf_t now = get_transform(m, link_id);
                double e[6];
                for (int k = 0; k < 3; ++k) e[k] = M(tgt, k, 3) - M(now, k, 3);
                if (prm->with_rot == 2) { /* the reference's f_objective (src/inverse_kinematics.jl:38-50) */
                    double rt[3], rn[3];
                    rpy_of(&tgt, rt);
                    rpy_of(&now, rn);
                    for (int k = 0; k < 3; ++k) {
                        const double d = rt[k] - rn[k]; /* wrapped to (-pi, pi] */
                        e[3 + k] = d - 6.283185307179586476925286766559 * rint(d * 0.15915494309189533576888376337251);
                    }
                } else if (prm->with_rot) {
                    rot_error(&tgt, &now, e + 3);
                }
                ep = sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
                er = prm->with_rot ? sqrt(e[3] * e[3] + e[4] * e[4] + e[5] * e[5]) : 0.0;
                if ((ep < prm->tol_pos && er < prm->tol_rot) || it >= prm->max_iters) break;
                if (attempt_len > 0 && it > 0 && it % attempt_len == 0) {
                    /* restart: relevant joints re-drawn within limits (U[-pi, pi] if unbounded), base reset */
                    const int32_t att = it / attempt_len;
                    for (int32_t c = 0; c < ndof; ++c) {
                        if (c < n_q && or_is_relevant(m, qids[c], link_id)) {
                            double l = lo[c], h = hi[c];
                            if (!isfinite(l) || !isfinite(h)) { l = -3.14159265358979323846; h = 3.14159265358979323846; }
                            a[c] = l + (h - l) * or_ik_seed_u01(prm->seed, i, att, c);
                        } else {
                            a[c] = a0[c];
                        }
                        held[c] = 0;
                    }
                    continue;
                }
                memset(J, 0, sizeof(double) * 6 * ndof);
                or_get_jacobian(m, link_id, n_q, qids, prm->with_rot != 0, prm->with_rot == 2, J);
                double dq[64], mx = 0;
                /* active set: joints held[k] (on a limit, pushed further out by the previous
                 * iteration's direction) are dropped from this solve (columns zeroed); every joint's
                 * unconstrained direction J_k^T y decides the set of the next iteration */
                {
                    double A[36], y[6];
                    const double lam2 = prm->lambda * prm->lambda + prm->damp_err * (ep * ep + er * er);
                    for (int r = 0; r < rows; ++r) y[r] = e[r];
                    for (int32_t k = 0; k < ndof; ++k)
                        for (int r = 0; r < rows; ++r) Jw[r + rows * k] = held[k] ? 0.0 : J[r + rows * k];
                    for (int c = 0; c < rows; ++c)
                        for (int r = 0; r < rows; ++r) {
                            double s = 0;
                            for (int32_t k = 0; k < ndof; ++k) s += Jw[r + rows * k] * Jw[c + rows * k];
                            A[r + rows * c] = s + (r == c ? lam2 : 0.0);
                        }
                    chol_solve(A, rows, y);
                    for (int32_t k = 0; k < ndof; ++k) {
                        double s = 0;
                        for (int r = 0; r < rows; ++r) s += J[r + rows * k] * y[r];
                        dq[k] = held[k] ? 0.0 : s;
                        held[k] = (a[k] <= lo[k] && s < 0) || (a[k] >= hi[k] && s > 0);
                        if (fabs(dq[k]) > mx) mx = fabs(dq[k]);
                    }
                }
                double sc = mx > prm->max_step ? prm->max_step / mx : 1.0;
                for (int32_t k = 0; k < ndof; ++k) {
                    double v = a[k] + sc * dq[k];
                    a[k] = v < lo[k] ? lo[k] : (v > hi[k] ? hi[k] : v);
                }
            }
            for (int32_t c = 0; c < ndof; ++c) q[c * ldq + i] = a[c];
            if (!(ep < prm->tol_pos && er < prm->tol_rot)) it = prm->max_iters + 1; /* not converged */
            if (iters_out) iters_out[i] = it;
            if (err_out) { err_out[i] = ep; err_out[n + i] = er; }
        }
        free(a); free(J); free(Jw); free(lo); free(hi);
        or_mech_destroy(m);
    }
}

/* ------------------------------------------------------------------ */
/* SDF + swept-sphere collision (src/sdf.jl, src/collision.jl)          */
/* ------------------------------------------------------------------ */
static tf_t tf_inv(const tf_t* t) { /* src/transform.jl:62-65 */
    tf_t r = tf_identity();
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M(r, i, j) = M(*t, j, i);
    for (int i = 0; i < 3; ++i)
        M(r, i, 3) = -(M(r, i, 0) * M(*t, 0, 3) + M(r, i, 1) * M(*t, 1, 3) + M(r, i, 2) * M(*t, 2, 3));
    return r;
}

or_union_sdf* or_sdf_create(int32_t n, const double* poses16, const double* widths3) {
    or_union_sdf* s = (or_union_sdf*)calloc(1, sizeof(or_union_sdf));
    s->n_boxes = n;
    s->inv_pose = (double*)malloc(sizeof(double) * 16 * (n + 1));
    s->width = (double*)malloc(sizeof(double) * 3 * (n + 1));
    for (int32_t k = 0; k < n; ++k) {
        tf_t t; memcpy(t.m, poses16 + 16 * k, sizeof t.m);
        tf_t r = tf_inv(&t);
        memcpy(s->inv_pose + 16 * k, r.m, sizeof r.m);
        memcpy(s->width + 3 * k, widths3 + 3 * k, sizeof(double) * 3);
    }
    return s;
}

void or_sdf_destroy(or_union_sdf* s) {
    if (!s) return;
    free(s->inv_pose); free(s->width); free(s);
}

double or_box_sdf(const or_union_sdf* s, int32_t k, const double* p) {
    const double* T = s->inv_pose + 16 * k;
    double q[3], mx = -INFINITY, nrm = 0;
    for (int i = 0; i < 3; ++i) {
        /* inv_pose * p = translation + rotation * p (src/transform.jl:39-41) */
        double l = T[12 + i] + (T[i] * p[0] + T[4 + i] * p[1] + T[8 + i] * p[2]);
        q[i] = fabs(l) - 0.5 * s->width[3 * k + i];
        if (q[i] > mx) mx = q[i];
        double c = q[i] > 0 ? q[i] : 0.0;
        nrm += c * c;
    }
    return sqrt(nrm) + (mx < 0 ? mx : 0.0);
}

double or_union_sdf_value(const or_union_sdf* s, const double* p, int32_t* argmin) {
    double best = INFINITY;
    int32_t bi = 0;
    for (int32_t k = 0; k < s->n_boxes; ++k) {
        double v = or_box_sdf(s, k, p);
        if (v < best) { best = v; bi = k; }  /* argmin: first minimum */
    }
    if (argmin) *argmin = bi;
    return best;
}

void or_union_sdf_gradient(const or_union_sdf* s, const double* p, double* g) {
    int32_t k;
    double v0 = or_union_sdf_value(s, p, &k);
    const double eps = 1e-7;
    for (int i = 0; i < 3; ++i) {
        double t[3] = {p[0], p[1], p[2]};
        t[i] += eps;
        g[i] = (or_box_sdf(s, k, t) - v0) / eps;
    }
}

void or_coll_batch(const or_mech* proto, const or_union_sdf* sdf, int64_t n, const double* q, int64_t ldq,
                   int32_t n_q, const int32_t* qids, int32_t n_sph, const int32_t* sph, const double* radii,
                   double trunc, double* dists, int64_t ldd, double* grads, int64_t ldg, int32_t n_threads) {
    int nt = nthreads_of(n_threads);
    int32_t ncolq = n_q + (proto->with_base ? 3 : 0);
#pragma omp parallel num_threads(nt)
    {
        or_mech* m = or_mech_clone(proto);
        double* a = (double*)malloc(sizeof(double) * (ncolq + 1));
        double* J = (double*)malloc(sizeof(double) * 3 * (ncolq + 1));
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            for (int32_t c = 0; c < ncolq; ++c) a[c] = q[c * ldq + i];
            or_set_joint_angles(m, n_q, qids, a);
            for (int32_t k = 0; k < n_sph; ++k) {
                tf_t t = get_transform(m, sph[k]);
                double p[3] = {M(t, 0, 3), M(t, 1, 3), M(t, 2, 3)};
                double d0 = or_union_sdf_value(sdf, p, NULL) - radii[k];
                if (d0 > trunc) {
                    dists[(size_t)k * ldd + i] = trunc;
                    if (grads)
                        for (int32_t c = 0; c < ncolq; ++c) grads[((size_t)k * ncolq + c) * ldg + i] = 0.0;
                    continue;
                }
                dists[(size_t)k * ldd + i] = d0;
                if (grads) {
                    double g[3];
                    or_union_sdf_gradient(sdf, p, g);
                    memset(J, 0, sizeof(double) * 3 * ncolq);
                    or_get_jacobian(m, sph[k], n_q, qids, 0, 0, J);
                    for (int32_t c = 0; c < ncolq; ++c)
                        grads[((size_t)k * ncolq + c) * ldg + i] = g[0] * J[3 * c] + g[1] * J[3 * c + 1] + g[2] * J[3 * c + 2];
                }
            }
        }
        free(a); free(J);
        or_mech_destroy(m);
    }
}

/* ---- build-defined collision-aware IK (kin_ik_coll_batch), restated for parity ----
 * Stage 2 of inverse_kinematics!(m, link, joints, target, sscc, sdf) (src/inverse_kinematics.jl:1-21)
 * as the GPU kernel does it (kinhip_ikt_dev.h): per iteration the pose residual e (with_rot as in
 * or_ik_dls_batch) and, for every sphere with d_k < margin + band, the IneqConst row a_k = grad sdf^T J_k
 * (analytic gradient of the argmin box); one damped Gauss-Newton step on the normal equations
 *   (J^T J + w^2 sum a_k^T a_k + lambda^2 I) dq = J^T e + w^2 sum a_k^T (margin + band - d_k)
 * over the free variables -- the joints that move the target link or a sphere link (spheres may hang off
 * any chain of the tree) and the base -- joints held out while on a limit and pushed outward (by the last
 * step, or by the right-hand side while held), |dq|_inf <= max_step, clamp; converged when |dp| < tol_pos,
 * |rot| < tol_rot and every d_k >= margin - feas.  Restarts as or_ik_dls_batch (every free joint
 * re-drawn).  Not converged: the attempt whose end state has the lowest merit
 * |dp|^2 + |rot|^2 + w^2 max(0, margin - min d)^2 (NaN = worst; ties: the earlier attempt).
 * sdfs (optional): one union per target (boxes of a scene mechanism at that target's scene state). */
static void box_gradient_analytic(const or_union_sdf* s, int32_t k, const double* p, double g[3]) {
    const double* T = s->inv_pose + 16 * k;
    double l[3], q[3], gl[3];
    for (int i = 0; i < 3; ++i) {
        l[i] = T[12 + i] + (T[i] * p[0] + T[4 + i] * p[1] + T[8 + i] * p[2]);
        q[i] = fabs(l[i]) - 0.5 * s->width[3 * k + i];
    }
    double mx = q[0] > q[1] ? q[0] : q[1];
    mx = q[2] > mx ? q[2] : mx;
    if (mx > 0) {
        double o[3], nn = 0;
        for (int i = 0; i < 3; ++i) { o[i] = q[i] > 0 ? q[i] : 0.0; nn += o[i] * o[i]; }
        nn = sqrt(nn);
        for (int i = 0; i < 3; ++i) gl[i] = (l[i] < 0 ? -o[i] : o[i]) / nn;
    } else {
        int im = (q[0] >= q[1] && q[0] >= q[2]) ? 0 : (q[1] >= q[2] ? 1 : 2);
        for (int i = 0; i < 3; ++i) gl[i] = i == im ? (l[i] < 0 ? -1.0 : 1.0) : 0.0;
    }
    for (int j = 0; j < 3; ++j) g[j] = T[4 * j] * gl[0] + T[4 * j + 1] * gl[1] + T[4 * j + 2] * gl[2];
}

void or_ik_coll_batch(const or_mech* proto, const or_union_sdf* sdf, int64_t n, double* q, int64_t ldq, int32_t n_q,
                      const int32_t* qids, int32_t link_id, const double* target, int64_t ldt, const or_ik_params* prm,
                      const double* cprm, int32_t n_sph, const int32_t* sph, const double* radii,
                      const or_union_sdf* const* sdfs, const double* q_alt, int32_t* iters_out, double* err_out,
                      int32_t n_threads) {
    int nt = nthreads_of(n_threads);
    const int32_t nd = n_q + (proto->with_base ? 3 : 0);
    const int rows = prm->with_rot ? 6 : 3;
    const double margin = cprm[0], band = cprm[1], w2 = cprm[2] * cprm[2], feas = cprm[3];
#pragma omp parallel num_threads(nt)
    {
        or_mech* m = or_mech_clone(proto);
        double* a = (double*)malloc(sizeof(double) * (nd + 1));
        double* J = (double*)malloc(sizeof(double) * 6 * (nd + 1));
        double* J3 = (double*)malloc(sizeof(double) * 3 * (nd + 1));
        double* A = (double*)malloc(sizeof(double) * (nd + 1) * (nd + 1));
        double* bv = (double*)malloc(sizeof(double) * (nd + 1));
        double* y = (double*)malloc(sizeof(double) * (nd + 1));
        double* av = (double*)malloc(sizeof(double) * (nd + 1));
        double* lo = (double*)malloc(sizeof(double) * (nd + 1));
        double* hi = (double*)malloc(sizeof(double) * (nd + 1));
        double* best = (double*)malloc(sizeof(double) * (nd + 1));
        int* rel = (int*)malloc(sizeof(int) * (nd + 1));
        for (int32_t c = 0; c < nd; ++c) {
            if (c >= n_q) {
                rel[c] = 1;
            } else {
                const int32_t j = qids[c];
                int r = m->jtype[j - 1] != OR_FIXED && or_is_relevant(m, j, link_id);
                for (int32_t k = 0; k < n_sph && !r; ++k) r = m->jtype[j - 1] != OR_FIXED && or_is_relevant(m, j, sph[k]);
                /* a repeated joint keeps its last column (set_joint_angles) */
                for (int32_t c2 = c + 1; c2 < n_q && r; ++c2) if (qids[c2] == j) r = 0;
                rel[c] = r;
            }
            lo[c] = c < n_q && rel[c] ? m->jlower[qids[c] - 1] : -INFINITY;
            hi[c] = c < n_q && rel[c] ? m->jupper[qids[c] - 1] : INFINITY;
        }
#pragma omp for schedule(static)
        for (int64_t i = 0; i < n; ++i) {
            const or_union_sdf* sd = sdfs ? sdfs[i] : sdf;
            tf_t tgt = tf_identity();
            for (int k = 0; k < 12; ++k) tgt.m[(k / 3) * 4 + (k % 3)] = target[(size_t)k * ldt + i];
            double trpy[3];
            rpy_of(&tgt, trpy);
            for (int32_t c = 0; c < nd; ++c) a[c] = q[c * ldq + i];
            double a0[64];
            int held[64];
            for (int32_t c = 0; c < nd; ++c) { a0[c] = a[c]; held[c] = 0; best[c] = a[c]; }
            const int32_t attempt_len = prm->restarts > 0 ? prm->max_iters / (prm->restarts + 1) : 0;
            int32_t it = 0;
            int conv = 0;
            double ep = 0, er = 0, dmin = INFINITY;
            double best_m = INFINITY, bep = 0, ber = 0, bdm = 0;
            int have_best = 0;
            for (;; ++it) {
                or_set_joint_angles(m, n_q, qids, a);
                memset(A, 0, sizeof(double) * nd * nd);
                memset(bv, 0, sizeof(double) * nd);
                dmin = INFINITY;
                for (int32_t k = 0; k < n_sph; ++k) {
                    tf_t t = get_transform(m, sph[k]);
                    double p[3] = {M(t, 0, 3), M(t, 1, 3), M(t, 2, 3)};
                    int32_t kb = 0;
                    const double d = or_union_sdf_value(sd, p, &kb) - radii[k];
                    if (d < dmin) dmin = d;
                    const double viol = margin + band - d;
                    if (viol > 0) {
                        double g[3];
                        box_gradient_analytic(sd, kb, p, g);
                        memset(J3, 0, sizeof(double) * 3 * nd);
                        or_get_jacobian(m, sph[k], n_q, qids, 0, 0, J3);
                        for (int32_t c = 0; c < nd; ++c) av[c] = g[0] * J3[3 * c] + g[1] * J3[3 * c + 1] + g[2] * J3[3 * c + 2];
                        for (int32_t r = 0; r < nd; ++r) {
                            bv[r] += w2 * av[r] * viol;
                            for (int32_t c = 0; c < nd; ++c) A[r + nd * c] += w2 * av[r] * av[c];
                        }
                    }
                }
                tf_t now = get_transform(m, link_id);
                double e[6];
                for (int k = 0; k < 3; ++k) e[k] = M(tgt, k, 3) - M(now, k, 3);
                if (prm->with_rot == 2) {
                    double rn[3];
                    rpy_of(&now, rn);
                    for (int k = 0; k < 3; ++k) {
                        const double dd = trpy[k] - rn[k];
                        e[3 + k] = dd - 6.283185307179586476925286766559 * rint(dd * 0.15915494309189533576888376337251);
                    }
                } else if (prm->with_rot) {
                    rot_error(&tgt, &now, e + 3);
                }
                ep = sqrt(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
                er = prm->with_rot ? sqrt(e[3] * e[3] + e[4] * e[4] + e[5] * e[5]) : 0.0;
                if (ep < prm->tol_pos && er < prm->tol_rot && dmin >= margin - feas) { conv = 1; break; }
                const int last = it >= prm->max_iters;
                const int over = !last && attempt_len > 0 && it > 0 && it % attempt_len == 0;
                if (last || over) {  /* an attempt ends: keep its end state if it is the best so far */
                    const double vm = margin - dmin > 0 ? margin - dmin : 0.0;
                    double mr = w2 * vm * vm + (ep * ep + er * er);
                    if (mr != mr) mr = INFINITY;
                    if (mr < best_m || !have_best) {
                        best_m = mr; have_best = 1;
                        for (int32_t c = 0; c < nd; ++c) best[c] = a[c];
                        bep = ep; ber = er; bdm = dmin;
                    }
                    if (last) break;
                    const int32_t att = it / attempt_len;
                    for (int32_t c = 0; c < nd; ++c) {
                        if (q_alt && (c >= n_q || (att == 1 && rel[c]))) {
                            /* kin_ik_coll_batch_alt: attempt 1 from the second start, every restart's base */
                            a[c] = q_alt[c * ldq + i];
                        } else if (c < n_q && rel[c]) {
                            double l = lo[c], h = hi[c];
                            if (!isfinite(l) || !isfinite(h)) { l = -3.14159265358979323846; h = 3.14159265358979323846; }
                            a[c] = l + (h - l) * or_ik_seed_u01(prm->seed, i, att, c);
                        } else {
                            a[c] = a0[c];
                        }
                        held[c] = 0;
                    }
                    continue;
                }
                memset(J, 0, sizeof(double) * 6 * nd);
                or_get_jacobian(m, link_id, n_q, qids, prm->with_rot != 0, prm->with_rot == 2, J);
                for (int32_t r = 0; r < nd; ++r) {
                    for (int k = 0; k < rows; ++k) bv[r] += J[k + rows * r] * e[k];
                    for (int32_t c = 0; c < nd; ++c) {
                        double s2 = 0;
                        for (int k = 0; k < rows; ++k) s2 += J[k + rows * r] * J[k + rows * c];
                        A[r + nd * c] += s2;
                    }
                }
                for (int32_t r = 0; r < nd; ++r) {
                    const int fr = rel[r] && !held[r];
                    for (int32_t c = 0; c < nd; ++c)
                        if (c != r && (!fr || !(rel[c] && !held[c]))) A[r + nd * c] = 0.0;
                    A[r + nd * r] = fr ? A[r + nd * r] + prm->lambda * prm->lambda : 1.0;
                    y[r] = fr ? bv[r] : 0.0;
                }
                chol_solve(A, nd, y);
                double mx = 0;
                for (int32_t c = 0; c < nd; ++c) {
                    if (c < n_q && rel[c]) {
                        const double dir = held[c] ? bv[c] : y[c];
                        const int nh = (a[c] <= lo[c] && dir < 0) || (a[c] >= hi[c] && dir > 0);
                        if (held[c]) y[c] = 0.0;
                        held[c] = nh;
                    }
                    if (fabs(y[c]) > mx) mx = fabs(y[c]);
                }
                const double sc = mx > prm->max_step ? prm->max_step / mx : 1.0;
                for (int32_t c = 0; c < nd; ++c) {
                    if (!rel[c]) continue;
                    const double v = a[c] + sc * y[c];
                    a[c] = v < lo[c] ? lo[c] : (v > hi[c] ? hi[c] : v);
                }
            }
            if (!conv) {
                for (int32_t c = 0; c < nd; ++c) a[c] = best[c];
                ep = bep; er = ber; dmin = bdm;
            }
            for (int32_t c = 0; c < nd; ++c) q[c * ldq + i] = a[c];
            if (iters_out) iters_out[i] = conv ? it : prm->max_iters + 1;
            if (err_out) { err_out[i] = ep; err_out[n + i] = er; err_out[2 * n + i] = dmin; }
        }
        free(a); free(J); free(J3); free(A); free(bv); free(y); free(av); free(lo); free(hi); free(best); free(rel);
        or_mech_destroy(m);
    }
}
