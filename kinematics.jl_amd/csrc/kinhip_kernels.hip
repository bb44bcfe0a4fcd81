// kinhip_kernels.hip -- gfx950 (MI355X / CDNA4) kernels of the batched
// kinematics engine.  Compiled only for --offload-arch=gfx950.
//
// Reference semantics (HiroIshida/Kinematics.jl):
//   k_fk        get_transform over many links + get_jacobian!  (src/algorithm.jl:1-106,
//               joint_transform src/mechanism.jl:90-103, rpy src/transform.jl:45-48)
//   k_ik_dls    batched damped-least-squares replacement of the SLSQP loop of
//               inverse_kinematics! (src/inverse_kinematics.jl:23-64), build-defined
//   k_nakamura  point_inverse_kinematics_nakamura (src/algorithm.jl:116-131)
//
// Execution model: one configuration per lane (wave64).  Joint angles, poses
// and Jacobians are SoA with the configuration index fastest, so every load
// and store of a wave touches 64 consecutive elements (256 B fp32 / 512 B
// fp64).  The staged program (kinhip_prog.h) is identical for every lane: its
// fields are read with uniform addresses (scalar loads through the scalar
// cache), and its control flow is wave-uniform.  The root -> Jacobian-link
// chain ("phase A", <= MAXA steps) is fully unrolled so that the per-joint
// world origins/axes the Jacobian needs stay in registers; other links are
// evaluated by a uniform loop that branches through per-lane LDS slots.
// No MFMA: 3x4 rigid products are not a dense contraction; the kernels are
// HBM-bound at the sizes of BASELINE.json (roofline).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>

#include <algorithm>

#include "kinhip_internal.h"




namespace kinhip {
namespace {

template <typename T>
struct Fr {
    T r[9];  // row-major rotation
    T t[3];
};

// sin/cos of joint angles.  The library sincos carries a Payne-Hanek
// reduction for huge arguments that, inlined once per joint, dominates the
// kernel's code and register budget.  Joint angles are small, so: Cody-Waite
// reduction by pi/2 with FMA-split constants, minimax kernels on [-pi/4, pi/4]
// (Cephes sinf/cosf for fp32, fdlibm __kernel_sin/__kernel_cos for fp64), and
// the library call kept only behind a rarely taken |x| bound.
__device__ __noinline__ void sincos_slow(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ __noinline__ void sincos_slow(double x, double* s, double* c) { sincos(x, s, c); }

__device__ __forceinline__ void sincos_t(float x, float* s, float* c) {
    if (__builtin_expect(!(fabsf(x) < 8192.0f), 0)) {
        sincos_slow(x, s, c);
        return;
    }
    const float j = rintf(x * 0.636619772367581343f);
    float r = fmaf(-j, 1.57079637050628662109375f, x);
    r = fmaf(-j, -4.37113900018624283e-8f, r);
    const float z = r * r;
    const float sp = fmaf(r * z, fmaf(z, fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), r);
    const float cp = fmaf(z * z, fmaf(z, fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f),
                          fmaf(-0.5f, z, 1.0f));
    const int qd = (int)j & 3;
    const float ss = (qd & 1) ? cp : sp, cc = (qd & 1) ? sp : cp;
    *s = (qd & 2) ? -ss : ss;
    *c = ((qd + 1) & 2) ? -cc : cc;
}

__device__ __forceinline__ void sincos_t(double x, double* s, double* c) {
    if (__builtin_expect(!(fabs(x) < 1048576.0), 0)) {
        sincos_slow(x, s, c);
        return;
    }
    const double j = rint(x * 0.63661977236758134308);
    double r = fma(-j, 1.57079632679489655800e+00, x);
    r = fma(-j, 6.12323399573676603587e-17, r);
    r = fma(-j, -1.49738490485916983e-33, r);
    const double z = r * r;
    const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                                  2.75573137070700676789e-06),
                                        -1.98412698298579493134e-04),
                              8.33333333332248946124e-03),
                          -1.66666666666666324348e-01);
    const double sp = fma(r * z, ps, r);
    const double pc = z * fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                                   -2.75573143513906633035e-07),
                                         2.48015872894767294178e-05),
                               -1.38888888888741095749e-03),
                           4.16666666666666019037e-02);
    const double hz = 0.5 * z;
    const double w = 1.0 - hz;
    const double cp = w + (((1.0 - w) - hz) + z * pc);
    const int qd = (int)(long long)j & 3;
    const double ss = (qd & 1) ? cp : sp, cc = (qd & 1) ? sp : cp;
    *s = (qd & 2) ? -ss : ss;
    *c = ((qd + 1) & 2) ? -cc : cc;
}
__device__ __forceinline__ float atan2_t(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double atan2_t(double y, double x) { return atan2(y, x); }
__device__ __forceinline__ float sqrt_t(float x) { return sqrtf(x); }
__device__ __forceinline__ double sqrt_t(double x) { return sqrt(x); }

// SoA addressing: element `row` of a [rows][ld] array for this lane.  Each
// row gets a wave-uniform buffer descriptor (SGPRs: base = row pointer) and
// every load/store uses the same 32-bit lane byte offset (one VGPR), i.e.
// `buffer_load/store_dword v, v_off, s[rsrc], 0 offen` -- no 64-bit per-access
// address arithmetic in VGPRs.  The launcher splits batches (kChunk) so lane
// byte offsets stay below 2^31.  KINHIP_STORE_AUX selects the cache policy of
// the output stream (0 = default, 2 = nt: +10% on the FK+J stream, A/B in
// profiles/r01_ab_variants.txt).
#ifndef KINHIP_STORE_AUX
#define KINHIP_STORE_AUX 2
#endif
typedef unsigned int u32x2 __attribute__((__vector_size__(8)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float ld_soa(const float* __restrict__ base, int64_t row, int64_t ld, uint32_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(row_rsrc(base + row * ld), (int)off, 0, 0));
}
__device__ __forceinline__ double ld_soa(const double* __restrict__ base, int64_t row, int64_t ld, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(row_rsrc(base + row * ld), (int)off, 0, 0));
}
__device__ __forceinline__ void st_soa(float* __restrict__ base, int64_t row, int64_t ld, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), row_rsrc(base + row * ld), (int)off, 0, KINHIP_STORE_AUX);
}
__device__ __forceinline__ void st_soa(double* __restrict__ base, int64_t row, int64_t ld, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), row_rsrc(base + row * ld), (int)off, 0,
                                          KINHIP_STORE_AUX);
}

template <typename T>
__device__ __forceinline__ void set_identity(Fr<T>& f) {
#pragma unroll
    for (int k = 0; k < 9; ++k) f.r[k] = (k % 4 == 0) ? T(1) : T(0);
    f.t[0] = f.t[1] = f.t[2] = T(0);
}

// f <- f * F   (F: row-major 3x4 in uniform memory)
template <typename T>
__device__ __forceinline__ void mul_rigid(Fr<T>& f, const T* __restrict__ F) {
    const T F0 = F[0], F1 = F[1], F2 = F[2], F3 = F[3];
    const T F4 = F[4], F5 = F[5], F6 = F[6], F7 = F[7];
    const T F8 = F[8], F9 = F[9], F10 = F[10], F11 = F[11];
    Fr<T> g;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const T a = f.r[3 * i], b = f.r[3 * i + 1], c = f.r[3 * i + 2];
        g.r[3 * i + 0] = fma(a, F0, fma(b, F4, c * F8));
        g.r[3 * i + 1] = fma(a, F1, fma(b, F5, c * F9));
        g.r[3 * i + 2] = fma(a, F2, fma(b, F6, c * F10));
        g.t[i] = fma(a, F3, fma(b, F7, fma(c, F11, f.t[i])));
    }
    f = g;
}

template <typename T>
__device__ __forceinline__ void mul_rigid_regs(Fr<T>& out, const Fr<T>& f, const T (&F)[12]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const T a = f.r[3 * i], b = f.r[3 * i + 1], c = f.r[3 * i + 2];
        out.r[3 * i + 0] = fma(a, F[0], fma(b, F[4], c * F[8]));
        out.r[3 * i + 1] = fma(a, F[1], fma(b, F[5], c * F[9]));
        out.r[3 * i + 2] = fma(a, F[2], fma(b, F[6], c * F[10]));
        out.t[i] = fma(a, F[3], fma(b, F[7], fma(c, F[11], f.t[i])));
    }
}

// joint motion in the canonical frame (axis = local z), branch-free in the
// joint kind: revolute -> (c, s, 0), prismatic -> (1, 0, scale*q), none -> (1, 0, 0)
template <typename T>
__device__ __forceinline__ void motion(Fr<T>& f, int32_t kind, int32_t flags, T scale, T qv) {
    const bool rev = kind == MOT_REV;
    T th = rev ? qv : T(0);
    if (flags & SF_SCALE) {  // UnitQuaternion normalisation of a non-unit axis
        T sh, ch;
        sincos_t(T(0.5) * qv, &sh, &ch);
        th = T(2) * atan2_t(scale * sh, ch);
    }
    T s, c;
    sincos_t(th, &s, &c);
    const T d = (kind == MOT_PRISM) ? scale * qv : T(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const T a = f.r[3 * i], b = f.r[3 * i + 1];
        f.r[3 * i] = fma(a, c, b * s);
        f.r[3 * i + 1] = fma(b, c, -(a * s));
        f.t[i] = fma(f.r[3 * i + 2], d, f.t[i]);
    }
}

template <typename T>
__device__ __forceinline__ void base_frame(Fr<T>& f, T bx, T by, T th) {  // src/transform.jl:33-37
    set_identity(f);
    T s, c;
    sincos_t(th, &s, &c);
    f.r[0] = c; f.r[1] = -s;
    f.r[3] = s; f.r[4] = c;
    f.t[0] = bx; f.t[1] = by;
}

// Output sink: runs of consecutive SoA rows of one array (a pose = 12 rows, a
// Jacobian column = 6 or 3 rows) for this lane's configuration, one 4/8-byte
// store per row.  (A 16-byte-per-lane variant staged through LDS measured 5%
// slower: this stream runs at the ceiling of its access pattern, see
// profiles/r01_store_probe.txt.)
template <typename T>
struct Sink {
    uint32_t off;  // lane byte offset

    template <int NR>
    __device__ __forceinline__ void rows(T* __restrict__ base, int64_t row0, int64_t ld, const T (&v)[NR],
                                         int nvalid) const {
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (k < nvalid) st_soa(base, row0 + k, ld, off, v[k]);
    }
};

// 3x4 column-major pose (k = row + 3*col) of output `o`: rows o*12 .. o*12+11
template <typename T>
__device__ __forceinline__ void store_pose(const Sink<T>& sk, T* __restrict__ poses, int64_t o, int64_t ld,
                                           const Fr<T>& L) {
    const T v[12] = {L.r[0], L.r[3], L.r[6], L.r[1], L.r[4], L.r[7], L.r[2], L.r[5], L.r[8], L.t[0], L.t[1], L.t[2]};
    sk.rows(poses, o * 12, ld, v, 12);
}

template <typename T>
__device__ __forceinline__ void link_frame(Fr<T>& L, const Fr<T>& C, bool has_x, const T* __restrict__ X) {
    if (has_x) {
        T Xr[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) Xr[k] = X[k];
        mul_rigid_regs(L, C, Xr);
    } else {
        L = C;
    }
}

template <typename T>
__device__ __forceinline__ void slot_store(T* slots, int slot, int B, int tid, const Fr<T>& f) {
    T* s = slots + (size_t)slot * 12 * B + tid;
#pragma unroll
    for (int k = 0; k < 9; ++k) s[k * B] = f.r[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) s[(9 + k) * B] = f.t[k];
}

template <typename T>
__device__ __forceinline__ void slot_load(const T* slots, int slot, int B, int tid, Fr<T>& f) {
    const T* s = slots + (size_t)slot * 12 * B + tid;
#pragma unroll
    for (int k = 0; k < 9; ++k) f.r[k] = s[k * B];
#pragma unroll
    for (int k = 0; k < 3; ++k) f.t[k] = s[(9 + k) * B];
}

// One phase-A step: C <- C F; record (o, z); motion.  Straight-line: padded
// steps are identities with scale 0, so records and motion need no branch.
template <typename T>
__device__ __forceinline__ void step_a(Fr<T>& f, const KStep<T>& st, T qv, T (&o)[3], T (&z)[3]) {
    mul_rigid(f, st.F);
    o[0] = f.t[0]; o[1] = f.t[1]; o[2] = f.t[2];  // _get_joint_axis, src/algorithm.jl:42-54
    const T sc = st.scale;
    z[0] = f.r[2] * sc; z[1] = f.r[5] * sc; z[2] = f.r[8] * sc;
    motion(f, st.kind, st.flags, sc, qv);
}

// One get_jacobian! column (src/algorithm.jl:65-81): revolute -> [z x (p - o); z or
// rpy_derivative!(z)], prismatic -> [z; untouched (zeros with get_jacobian)].
// Written to every column in the step's colmask.
template <typename T>
struct JacCtx {
    T* jac;
    int64_t ldj;
    const Sink<T>* sink;
    int rows;
    bool with_rot, zero, rpy;
    T px, py, pz;
    T k11, k12, k21, k22, k31, k32;  // rpy_derivative! coefficients
};

template <typename T>
__device__ __forceinline__ void emit_jcol(const JacCtx<T>& J, const KStep<T>& st, T ox, T oy, T oz, T zx, T zy,
                                          T zz) {
    T lin[3], ang[3];
    const bool prism = st.jkind == MOT_PRISM;
    if (prism) {
        lin[0] = zx; lin[1] = zy; lin[2] = zz;
        ang[0] = ang[1] = ang[2] = T(0);
    } else {
        const T dx = J.px - ox, dy = J.py - oy, dz = J.pz - oz;
        lin[0] = fma(zy, dz, -(zz * dy));
        lin[1] = fma(zz, dx, -(zx * dz));
        lin[2] = fma(zx, dy, -(zy * dx));
        if (J.rpy) {
            ang[0] = fma(J.k11, zx, J.k12 * zy);
            ang[1] = fma(J.k21, zx, J.k22 * zy);
            ang[2] = fma(J.k31, zx, fma(J.k32, zy, zz));
        } else {
            ang[0] = zx; ang[1] = zy; ang[2] = zz;
        }
    }
    const T v[6] = {lin[0], lin[1], lin[2], ang[0], ang[1], ang[2]};
    const int nv = (J.with_rot && (!prism || J.zero)) ? 6 : 3;
    uint64_t m = st.colmask;
    while (m) {
        const int c = __builtin_ctzll(m);
        m &= m - 1;
        J.sink->rows(J.jac, (int64_t)c * J.rows, J.ldj, v, nv);
    }
}

// Block -> configuration chunk.  Workgroups are dispatched round-robin over the
// 8 XCDs (block b on XCD b % 8); with KINHIP_XCD_REMAP each XCD instead takes
// one contiguous eighth of the batch, so its L2 and DRAM pages see sequential
// row segments rather than every eighth 1 KB piece.
#ifndef KINHIP_XCD_REMAP
#define KINHIP_XCD_REMAP 0
#endif
__device__ __forceinline__ uint32_t config_block() {
#if KINHIP_XCD_REMAP
    const uint32_t nb = gridDim.x, b = blockIdx.x, x = b & 7u, q = nb >> 3, r = nb & 7u;
    return x * q + (x < r ? x : r) + (b >> 3);
#else
    return blockIdx.x;
#endif
}

// --------------------------------------------------------------------------
// k_fk: batched get_transform (any set of links) + get_jacobian! of one link
// --------------------------------------------------------------------------
template <typename T, int MAXA>
__global__ __launch_bounds__(256) void k_fk(const KProg<T> P, const KStep<T>* __restrict__ S,
                                            const T* __restrict__ q, int64_t ldq, int64_t n,
                                            T* __restrict__ poses, int64_t ldp, T* __restrict__ jac,
                                            int64_t ldj) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* slots = reinterpret_cast<T*>(smem);
    const int B = blockDim.x, tid = threadIdx.x;
    const uint32_t i = config_block() * (uint32_t)B + tid;
    if (i >= (uint64_t)n) return;  // no block-wide barrier below: LDS slots are per lane
    const uint32_t off = i * (uint32_t)sizeof(T);
    Sink<T> sk;
    sk.off = off;

    const bool base = (P.flags & PF_BASE) != 0;
    T bx = T(0), by = T(0), bth = T(0);
    if (base) {
        bx = ld_soa(q, P.base_col, ldq, off);
        by = ld_soa(q, P.base_col + 1, ldq, off);
        bth = ld_soa(q, P.base_col + 2, ldq, off);
    }
    // every phase-A angle load issued up front (independent, coalesced)
    T qa[MAXA];
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const int32_t c = S[s].qcol;
        qa[s] = c >= 0 ? ld_soa(q, c, ldq, off) : T(0);
    }
    Fr<T> root;
    if (base) base_frame(root, bx, by, bth);
    else set_identity(root);

    Fr<T> f = root;
    // pre-motion world origin / axis of every phase-A joint, kept in registers
    // (a register-lighter form that re-derives them backwards with F^-1 measured
    // 20% slower: more VALU, profiles/r01_ab_variants.txt)
    T ro[MAXA][3], rz[MAXA][3];
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const KStep<T>& st = S[s];
        step_a(f, st, qa[s], ro[s], rz[s]);
        if (st.out >= 0) {
            Fr<T> L;
            link_frame(L, f, (st.flags & SF_HAS_X) != 0, st.X);
            store_pose(sk, poses, st.out, ldp, L);
        }
        if (st.save >= 0) slot_store(slots, st.save, B, tid, f);
    }

    if ((P.flags & PF_JAC) || P.spine_out >= 0) {
        Fr<T> L;
        link_frame(L, f, P.last_has_x != 0, P.Xlast);
        if (P.spine_out >= 0) store_pose(sk, poses, P.spine_out, ldp, L);
        if (P.flags & PF_JAC) {
            JacCtx<T> J;
            J.jac = jac; J.ldj = ldj; J.sink = &sk; J.rows = P.rows;
            J.with_rot = (P.flags & PF_WITH_ROT) != 0;
            J.zero = (P.flags & PF_ZERO) != 0;
            J.rpy = J.with_rot && (P.flags & PF_RPY);
            J.px = L.t[0]; J.py = L.t[1]; J.pz = L.t[2];
            J.k11 = J.k12 = J.k21 = J.k22 = J.k31 = J.k32 = T(0);
            if (J.rpy) {  // rpy_derivative! coefficients (src/algorithm.jl:56-63) from RotZYX(L)
                const T t1 = atan2_t(L.r[3], L.r[0]);
                T st1, ct1;
                sincos_t(t1, &st1, &ct1);
                const T t2 = atan2_t(-L.r[6], fma(L.r[3], st1, L.r[0] * ct1));
                T s2, c2, s3, c3;
                sincos_t(-t2, &s2, &c2);
                sincos_t(-t1, &s3, &c3);
                J.k11 = c3 / c2; J.k12 = -(s3 / c2);
                J.k21 = s3; J.k22 = c3;
                J.k31 = -(c3 * s2 / c2); J.k32 = s3 * s2 / c2;
            }
#pragma unroll
            for (int s = 0; s < MAXA; ++s)
                if (S[s].flags & SF_REC) emit_jcol(J, S[s], ro[s][0], ro[s][1], ro[s][2], rz[s][0], rz[s][1], rz[s][2]);
            const int rows = P.rows;
            if (J.zero) {
                const T z6[6] = {T(0), T(0), T(0), T(0), T(0), T(0)};
                uint64_t m = P.zmask;
                while (m) {
                    const int c = __builtin_ctzll(m);
                    m &= m - 1;
                    sk.rows(jac, (int64_t)c * rows, ldj, z6, rows);
                }
            }
            if (base) {  // src/algorithm.jl:98-105
                const T x = J.px - bx, y = J.py - by;
                const int64_t b0 = (int64_t)P.n_jac * rows;
                const T c0[6] = {T(1), T(0), T(0), T(0), T(0), T(0)};
                const T c1[6] = {T(0), T(1), T(0), T(0), T(0), T(0)};
                const T c2[6] = {-y, x, T(0), T(0), T(0), T(1)};
                sk.rows(jac, b0, ldj, c0, rows);
                sk.rows(jac, b0 + rows, ldj, c1, rows);
                sk.rows(jac, b0 + 2 * rows, ldj, c2, rows);
            }
        }
    }

    // phase B: the remaining links (uniform loop, LDS slots at branch points)
    for (int s = P.nA; s < P.nS; ++s) {
        const KStep<T>& st = S[s];
        const int32_t ld = st.load;
        if (ld == LOAD_ROOT) f = root;
        else if (ld >= 0) slot_load(slots, ld, B, tid, f);
        mul_rigid(f, st.F);
        if (st.kind != MOT_NONE) motion(f, st.kind, st.flags, st.scale, ld_soa(q, st.qcol, ldq, off));
        if (st.out >= 0) {
            Fr<T> L;
            link_frame(L, f, (st.flags & SF_HAS_X) != 0, st.X);
            store_pose(sk, poses, st.out, ldp, L);
        }
        if (st.save >= 0) slot_store(slots, st.save, B, tid, f);
    }
}

// --------------------------------------------------------------------------
// shared phase-A evaluator for the IK kernels: q per step in registers
// --------------------------------------------------------------------------
template <typename T, int MAXA>
__device__ __forceinline__ void chain_records(const KProg<T>& P, const KStep<T>* __restrict__ S,
                                              const Fr<T>& root, const T (&qs)[MAXA], Fr<T>& L,
                                              T (&ro)[MAXA][3], T (&rz)[MAXA][3]) {
    Fr<T> f = root;
#pragma unroll
    for (int s = 0; s < MAXA; ++s) step_a(f, S[s], qs[s], ro[s], rz[s]);
    link_frame(L, f, P.last_has_x != 0, P.Xlast);
}

// Jacobian column of phase-A step s (geometric; zero for non-recorded steps)
template <typename T, int ROWS>
__device__ __forceinline__ void jcol(const KStep<T>& st, const T (&o)[3], const T (&z)[3], const Fr<T>& L,
                                     T (&J)[ROWS]) {
    const T m = (st.flags & SF_REC) ? T(1) : T(0);
    if (st.jkind == MOT_PRISM) {
        J[0] = m * z[0]; J[1] = m * z[1]; J[2] = m * z[2];
        if constexpr (ROWS == 6) { J[3] = T(0); J[4] = T(0); J[5] = T(0); }
    } else {
        const T dx = L.t[0] - o[0], dy = L.t[1] - o[1], dz = L.t[2] - o[2];
        J[0] = m * fma(z[1], dz, -(z[2] * dy));
        J[1] = m * fma(z[2], dx, -(z[0] * dz));
        J[2] = m * fma(z[0], dy, -(z[1] * dx));
        if constexpr (ROWS == 6) { J[3] = m * z[0]; J[4] = m * z[1]; J[5] = m * z[2]; }
    }
}

// world rotation vector w with exp([w]) R = Rt  (log of Rt R^T)
template <typename T>
__device__ __forceinline__ void rot_error(const T (&Rt)[9], const T (&R)[9], T (&w)[3]) {
    T E[9];  // row-major E = Rt * R^T
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b)
            E[3 * a + b] = fma(Rt[3 * a], R[3 * b], fma(Rt[3 * a + 1], R[3 * b + 1], Rt[3 * a + 2] * R[3 * b + 2]));
    const T v0 = T(0.5) * (E[7] - E[5]);
    const T v1 = T(0.5) * (E[2] - E[6]);
    const T v2 = T(0.5) * (E[3] - E[1]);
    const T s = sqrt_t(v0 * v0 + v1 * v1 + v2 * v2);
    const T c = T(0.5) * (E[0] + E[4] + E[8] - T(1));
    const T th = atan2_t(s, c);
    if (s > T(1e-7)) {
        const T k = th / s;
        w[0] = v0 * k; w[1] = v1 * k; w[2] = v2 * k;
    } else if (c > T(0)) {
        w[0] = v0; w[1] = v1; w[2] = v2;
    } else {
        int b = 0;
        if (E[4] > E[0]) b = 1;
        if (E[8] > E[4 * b]) b = 2;
        T a[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) a[k] = T(0.5) * (E[3 * k + b] + E[3 * b + k]);
        a[b] = T(0.5) * (E[4 * b] + T(1));
        const T nn = sqrt_t(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
#pragma unroll
        for (int k = 0; k < 3; ++k) w[k] = a[k] / nn * th;
    }
}

template <typename T>
struct IkArgsT {
    int32_t max_iters;
    T lam2, tol_pos, tol_rot, max_step;
    int32_t attempt_len;  // 0: no restarts
    int32_t n_attempts;   // 1 + (max_iters - 1) / attempt_len (attempts the sequential schedule reaches)
    uint64_t seed;
    int64_t ibase;  // global index of this chunk's first configuration
};

// restart re-seed draw in [0, 1): identical to the oracle's or_ik_seed_u01
__device__ __forceinline__ double ik_seed_u01(uint64_t seed, int64_t i, int32_t attempt, int32_t col) {
    const uint64_t key = (uint64_t)i * 131ull + (uint64_t)attempt * 31ull + (uint64_t)col + 1ull;
    uint64_t z = seed + 0x9E3779B97F4A7C15ull * key + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}

// --------------------------------------------------------------------------
// k_ik_dls: batched damped least squares, dq = J^T (J J^T + lambda^2 I)^-1 e
//
// Restart schedule (kin_ik_params): attempt 0 starts from q0 and is checked at
// iterations 0..L; attempt k >= 1 starts from seeded random angles at
// iteration kL + 1 and ends at (k+1)L (the last one at max_iters); the answer
// is the first attempt that converges.  Attempts are independent, so G lanes
// of one wave share a target and run attempts slot, slot + G, ... side by side
// (G = 1: the plain sequential loop).  Each lane's arithmetic is exactly the
// sequential schedule's; a lane stops once a lower attempt of its target has
// converged, and the lowest converged attempt (else the last one) is written.
// Small batches (65k targets = one wave per SIMD) gain G x the parallelism.
// --------------------------------------------------------------------------
template <typename T, int MAXA>
__device__ __forceinline__ void ik_start_attempt(const KStep<T>* __restrict__ S, const IkArgsT<T>& a,
                                                 const T* __restrict__ q, int64_t ldq, uint32_t off, int64_t gi,
                                                 int att, T (&qs)[MAXA]) {
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const KStep<T>& st = S[s];
        const int32_t c = st.qcol;
        T v = c >= 0 ? ld_soa(q, c, ldq, off) : T(0);
        if (att > 0 && c >= 0) {
            if (st.flags & SF_REC) {
                double lo = (double)st.lo, hi = (double)st.hi;
                if (!isfinite(lo) || !isfinite(hi)) { lo = -3.14159265358979323846; hi = 3.14159265358979323846; }
                v = (T)(lo + (hi - lo) * ik_seed_u01(a.seed, gi, att, c));
            } else {
                v = fmin(fmax(v, st.lo), st.hi);  // attempt 0's first step has clamped it
            }
        }
        qs[s] = v;
    }
}

#ifndef KINHIP_IK_WAVES
#define KINHIP_IK_WAVES 1
#endif
template <typename T, int MAXA, int ROWS, int G>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KINHIP_IK_WAVES))) void k_ik_dls(const KProg<T> P, const KStep<T>* __restrict__ S,
                                                const IkArgsT<T> a, const T* __restrict__ tgt, int64_t ldt,
                                                T* __restrict__ q, int64_t ldq, int64_t n,
                                                int32_t* __restrict__ iters, T* __restrict__ err,
                                                int64_t lde) {
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t i = gt / G;  // target (lanes of one target are adjacent: same wave)
    const int slot = (int)(gt % G);
    const bool valid = i < (uint64_t)n;
    const uint32_t off = (valid ? i : 0u) * (uint32_t)sizeof(T);
    T Rt[9], pt[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) Rt[3 * r + c] = ld_soa(tgt, r + 3 * c, ldt, off);
        pt[r] = ld_soa(tgt, 9 + r, ldt, off);
    }
    const bool base = (P.flags & PF_BASE) != 0;
    T b0[3] = {T(0), T(0), T(0)};
    if (base)
        for (int k = 0; k < 3; ++k) b0[k] = ld_soa(q, P.base_col + k, ldq, off);
    const int64_t gi = a.ibase + (int64_t)i;
    const int L = a.attempt_len;

    int att = slot;
    bool done = !valid || att >= a.n_attempts;
    int res_att = INT_MAX;  // attempt at which this lane converged
    bool final_lane = false;
    T qs[MAXA], b[3] = {b0[0], b0[1], b0[2]};
    int it = att > 0 ? att * L + 1 : 0;
    ik_start_attempt<T, MAXA>(S, a, q, ldq, off, gi, att, qs);
    T ep = 0, er = 0;
    T ro[MAXA][3], rz[MAXA][3];
    for (;;) {
        if constexpr (G > 1) {  // lowest converged attempt of this target so far
            int gm = res_att;
#pragma unroll
            for (int w = 1; w < G; w <<= 1) gm = min(gm, __shfl_xor(gm, w, G));
            if (!done && gm < att) done = true;
        }
        if (__ballot(!done) == 0) break;  // wave-uniform exit: every lane finished or superseded
        if (done) continue;
        Fr<T> root, L_;
        if (base) base_frame(root, b[0], b[1], b[2]);
        else set_identity(root);
        chain_records<T, MAXA>(P, S, root, qs, L_, ro, rz);
        const Fr<T>& Lf = L_;
        T e[6];
        e[0] = pt[0] - Lf.t[0]; e[1] = pt[1] - Lf.t[1]; e[2] = pt[2] - Lf.t[2];
        ep = sqrt_t(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
        er = T(0);
        if constexpr (ROWS == 6) {
            T w[3];
            rot_error(Rt, Lf.r, w);
            e[3] = w[0]; e[4] = w[1]; e[5] = w[2];
            er = sqrt_t(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        }
        if (ep < a.tol_pos && er < a.tol_rot) {
            res_att = att;
            done = true;
            continue;
        }
        if (it >= a.max_iters) {  // only the last attempt gets here
            final_lane = true;
            done = true;
            continue;
        }
        if (L > 0 && it > 0 && it % L == 0) {  // attempt over: this lane's next one, if any
            att += G;
            if (att >= a.n_attempts) {
                done = true;
            } else {
                it = att * L + 1;
                ik_start_attempt<T, MAXA>(S, a, q, ldq, off, gi, att, qs);
                b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2];
            }
            continue;
        }

        T Jb[3][ROWS];
        if (base) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int r = 0; r < ROWS; ++r) Jb[k][r] = T(0);
            Jb[0][0] = T(1);
            Jb[1][1] = T(1);
            Jb[2][0] = -(Lf.t[1] - b[1]);
            Jb[2][1] = Lf.t[0] - b[0];
            if constexpr (ROWS == 6) Jb[2][5] = T(1);
        }
        // pass 0: every joint; pass 1 (lanes that need it): joints sitting on a
        // limit that the step pushes further out get weight 0 and the system is
        // re-solved (same rule as the oracle's or_ik_dls_batch)
        T w[MAXA];
#pragma unroll
        for (int s = 0; s < MAXA; ++s) w[s] = T(1);
        T dq[MAXA], db[3] = {T(0), T(0), T(0)};
        T mx = T(0);
        for (int pass = 0; pass < 2; ++pass) {
            // A = J W J^T + lambda^2 I  (lower triangle)
            T A[ROWS][ROWS];
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
#pragma unroll
                for (int c = 0; c < ROWS; ++c) A[r][c] = (r == c) ? a.lam2 : T(0);
#pragma unroll
            for (int s = 0; s < MAXA; ++s) {
                T J[ROWS];
                jcol<T, ROWS>(S[s], ro[s], rz[s], Lf, J);
#pragma unroll
                for (int r = 0; r < ROWS; ++r) J[r] *= w[s];
#pragma unroll
                for (int r = 0; r < ROWS; ++r)
#pragma unroll
                    for (int c = 0; c <= r; ++c) A[r][c] = fma(J[r], J[c], A[r][c]);
            }
            if (base) {
#pragma unroll
                for (int k = 0; k < 3; ++k)
#pragma unroll
                    for (int r = 0; r < ROWS; ++r)
#pragma unroll
                        for (int c = 0; c <= r; ++c) A[r][c] = fma(Jb[k][r], Jb[k][c], A[r][c]);
            }
            // Cholesky A = L L^T (in place, lower), then y = A^-1 e
#pragma unroll
            for (int j = 0; j < ROWS; ++j) {
                T d = A[j][j];
#pragma unroll
                for (int k = 0; k < j; ++k) d -= A[j][k] * A[j][k];
                d = sqrt_t(d);
                A[j][j] = d;
#pragma unroll
                for (int r = j + 1; r < ROWS; ++r) {
                    T sm = A[r][j];
#pragma unroll
                    for (int k = 0; k < j; ++k) sm -= A[r][k] * A[j][k];
                    A[r][j] = sm / d;
                }
            }
            T y[ROWS];
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                T sm = e[r];
#pragma unroll
                for (int k = 0; k < r; ++k) sm -= A[r][k] * y[k];
                y[r] = sm / A[r][r];
            }
#pragma unroll
            for (int r = ROWS - 1; r >= 0; --r) {
                T sm = y[r];
#pragma unroll
                for (int k = r + 1; k < ROWS; ++k) sm -= A[k][r] * y[k];
                y[r] = sm / A[r][r];
            }
            bool blocked = false;
            mx = T(0);
#pragma unroll
            for (int s = 0; s < MAXA; ++s) {
                T J[ROWS];
                jcol<T, ROWS>(S[s], ro[s], rz[s], Lf, J);
                T v = T(0);
#pragma unroll
                for (int r = 0; r < ROWS; ++r) v = fma(J[r], y[r], v);
                v *= w[s];
                dq[s] = v;
                if ((qs[s] <= S[s].lo && v < T(0)) || (qs[s] >= S[s].hi && v > T(0))) {
                    blocked = true;
                    w[s] = T(0);
                }
                mx = fmax(mx, fabs(v));
            }
            if (base) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    T v = T(0);
#pragma unroll
                    for (int r = 0; r < ROWS; ++r) v = fma(Jb[k][r], y[r], v);
                    db[k] = v;
                    mx = fmax(mx, fabs(v));
                }
            }
            if (!blocked) break;
        }
        const T sc = mx > a.max_step ? a.max_step / mx : T(1);
#pragma unroll
        for (int s = 0; s < MAXA; ++s) qs[s] = fmin(fmax(qs[s] + sc * dq[s], S[s].lo), S[s].hi);
        if (base)
            for (int k = 0; k < 3; ++k) b[k] = b[k] + sc * db[k];
        ++it;
    }
    bool writer = final_lane;
    if constexpr (G > 1) {
        int gm = res_att;
#pragma unroll
        for (int w = 1; w < G; w <<= 1) gm = min(gm, __shfl_xor(gm, w, G));
        writer = (gm != INT_MAX) ? (res_att == gm) : final_lane;
    } else {
        writer = valid;
    }
    if (!writer) return;
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const int32_t c = S[s].qcol;
        if (c >= 0) st_soa(q, c, ldq, off, qs[s]);
    }
    if (base)
        for (int k = 0; k < 3; ++k) st_soa(q, P.base_col + k, ldq, off, b[k]);
    if (iters) iters[i] = it;
    if (err) {
        st_soa(err, 0, lde, off, ep);
        st_soa(err, 1, lde, off, er);
    }
}

// --------------------------------------------------------------------------
// k_nakamura: point_inverse_kinematics_nakamura, 50 iterations
// --------------------------------------------------------------------------
template <typename T, int MAXA>
__global__ __launch_bounds__(256) void k_nakamura(const KProg<T> P, const KStep<T>* __restrict__ S,
                                                  const T* __restrict__ pts, int64_t ldpt, T* __restrict__ q,
                                                  int64_t ldq, int64_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)n) return;
    const uint32_t off = i * (uint32_t)sizeof(T);
    const T pd0 = ld_soa(pts, 0, ldpt, off), pd1 = ld_soa(pts, 1, ldpt, off), pd2 = ld_soa(pts, 2, ldpt, off);
    T qs[MAXA];
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const int32_t c = S[s].qcol;
        qs[s] = c >= 0 ? ld_soa(q, c, ldq, off) : T(0);
    }
    Fr<T> root;
    set_identity(root);
    T ro[MAXA][3], rz[MAXA][3];
    for (int it = 0; it < 50; ++it) {
        Fr<T> L;
        chain_records<T, MAXA>(P, S, root, qs, L, ro, rz);
        T a = 0, b = 0, c = 0, e = 0, f = 0, ii = 0;  // symmetric J J^T entries
#pragma unroll
        for (int s = 0; s < MAXA; ++s) {
            T J[3];
            jcol<T, 3>(S[s], ro[s], rz[s], L, J);
            a += J[0] * J[0]; b += J[0] * J[1]; c += J[0] * J[2];
            e += J[1] * J[1]; f += J[1] * J[2]; ii += J[2] * J[2];
        }
        // `jac * transpose(jac) .+ sr_weight`: +1.0 on EVERY entry (reference quirk)
        a += T(1); b += T(1); c += T(1); e += T(1); f += T(1); ii += T(1);
        const T d = b, g = c, h = f;  // symmetric
        const T A_ = e * ii - f * h, B_ = -(d * ii - f * g), C_ = d * h - e * g;
        const T det = a * A_ + b * B_ + c * C_;
        const T i00 = A_ / det, i01 = -(b * ii - c * h) / det, i02 = (b * f - c * e) / det;
        const T i10 = B_ / det, i11 = (a * ii - c * g) / det, i12 = -(a * f - c * d) / det;
        const T i20 = C_ / det, i21 = -(a * h - b * g) / det, i22 = (a * e - b * d) / det;
        const T dp0 = pd0 - L.t[0], dp1 = pd1 - L.t[1], dp2 = pd2 - L.t[2];
        const T y0 = i00 * dp0 + i01 * dp1 + i02 * dp2;
        const T y1 = i10 * dp0 + i11 * dp1 + i12 * dp2;
        const T y2 = i20 * dp0 + i21 * dp1 + i22 * dp2;
#pragma unroll
        for (int s = 0; s < MAXA; ++s) {
            T J[3];
            jcol<T, 3>(S[s], ro[s], rz[s], L, J);
            qs[s] += J[0] * y0 + J[1] * y1 + J[2] * y2;
        }
    }
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const int32_t c = S[s].qcol;
        if (c >= 0) st_soa(q, c, ldq, off, qs[s]);
    }
}

// --------------------------------------------------------------------------
// k_coll: compute_coll_dists_and_grads! (src/collision.jl:51-94) fused with FK:
// sphere centres from the phase-A frames, UnionSDF (min over BoxSDFs,
// src/sdf.jl:67-114) minus radius, gradient = grad_sdf^T J(3 x n) of the sphere
// link from the recorded joint origins / axes.  The SDF gradient is analytic
// (the reference takes a forward difference with eps 1e-7, src/sdf.jl:34-41;
// equal to it up to O(eps) away from the box's kinks).
// --------------------------------------------------------------------------
// Monotone surrogate of the box SDF, d*|d|: outside (max q > 0) |max(q,0)|^2,
// inside -(max q)^2.  The union takes the argmin of the surrogate (no square
// root per box; sqrt(fl(x*x)) == |x| recovers an inside distance exactly).
template <typename T>
__device__ __forceinline__ T box_key(T qx, T qy, T qz) {
    const T mx = fmax(qx, fmax(qy, qz));
    const T ox = fmax(qx, T(0)), oy = fmax(qy, T(0)), oz = fmax(qz, T(0));
    const T oo = fma(ox, ox, fma(oy, oy, oz * oz));
    return mx > T(0) ? oo : -(mx * mx);
}

template <typename T, bool GRAD>
__device__ __forceinline__ T union_sdf(const KBox<T>* __restrict__ boxes, const KAabb<T>* __restrict__ aabb, int na,
                                       int nb, T px, T py, T pz, T (&gw)[3]) {
    T best = T(INFINITY);
    int bk = 0;
    // uniform loops, box data through the scalar cache; argmin keeps the first minimum (Julia's argmin)
#pragma clang loop vectorize(disable) unroll_count(2)
    for (int k = 0; k < na; ++k) {  // axis-aligned boxes: no rotation
        const KAabb<T>& b = aabb[k];
        const T key = box_key(fabs(px - b.c[0]) - b.half[0], fabs(py - b.c[1]) - b.half[1],
                              fabs(pz - b.c[2]) - b.half[2]);
        if (GRAD) {
            if (key < best) {
                best = key;
                bk = k;
            }
        } else {
            best = fmin(best, key);
        }
    }
#pragma clang loop vectorize(disable)
    for (int k = na; k < nb; ++k) {
        const KBox<T>& b = boxes[k];
        const T qx = fabs(fma(b.inv[0], px, fma(b.inv[1], py, fma(b.inv[2], pz, b.inv[3])))) - b.half[0];
        const T qy = fabs(fma(b.inv[4], px, fma(b.inv[5], py, fma(b.inv[6], pz, b.inv[7])))) - b.half[1];
        const T qz = fabs(fma(b.inv[8], px, fma(b.inv[9], py, fma(b.inv[10], pz, b.inv[11])))) - b.half[2];
        const T key = box_key(qx, qy, qz);
        if (GRAD) {
            if (key < best) {
                best = key;
                bk = k;
            }
        } else {
            best = fmin(best, key);
        }
    }
    const T d = best > T(0) ? sqrt_t(best) : -sqrt_t(-best);
    if (GRAD) {  // analytic gradient of the argmin box, in its own frame, rotated to the world
        const KBox<T>& b = boxes[bk];
        T l[3], q[3], gl[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            l[i] = fma(b.inv[4 * i], px, fma(b.inv[4 * i + 1], py, fma(b.inv[4 * i + 2], pz, b.inv[4 * i + 3])));
            q[i] = fabs(l[i]) - b.half[i];
        }
        const T mx = fmax(q[0], fmax(q[1], q[2]));
        if (mx > T(0)) {  // outside: d = |max(q, 0)|
            const T o[3] = {fmax(q[0], T(0)), fmax(q[1], T(0)), fmax(q[2], T(0))};
            const T rn = T(1) / sqrt_t(o[0] * o[0] + o[1] * o[1] + o[2] * o[2]);
#pragma unroll
            for (int i = 0; i < 3; ++i) gl[i] = (l[i] < T(0) ? -o[i] : o[i]) * rn;
        } else {  // inside: d = max(q)
            const int im = (q[0] >= q[1] && q[0] >= q[2]) ? 0 : (q[1] >= q[2] ? 1 : 2);
#pragma unroll
            for (int i = 0; i < 3; ++i) gl[i] = (i == im) ? (l[i] < T(0) ? T(-1) : T(1)) : T(0);
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) gw[j] = fma(b.inv[j], gl[0], fma(b.inv[4 + j], gl[1], b.inv[8 + j] * gl[2]));
    }
    return d;
}

template <typename T, int MAXA, bool GRAD>
__device__ __forceinline__ void coll_spheres(int s_last, int k0, int k1, const Fr<T>& f, const KProg<T>& P,
                                             const KStep<T>* __restrict__ S, const KSphere<T>* __restrict__ sph,
                                             const KBox<T>* __restrict__ boxes, const KAabb<T>* __restrict__ aabb,
                                             int na, int nb, T trunc, T offs,
                                             const T (&ro)[MAXA][3], const T (&rz)[MAXA][3], T bx, T by,
                                             uint32_t off, T* __restrict__ dists, int64_t ldd,
                                             T* __restrict__ grads, int64_t ldg, T& dmin) {
    const int ndof = P.n_jac + ((P.flags & PF_BASE) ? 3 : 0);
    for (int k = k0; k < k1; ++k) {
        const KSphere<T>& sp = sph[k];
        const T px = fma(f.r[0], sp.c[0], fma(f.r[1], sp.c[1], fma(f.r[2], sp.c[2], f.t[0])));
        const T py = fma(f.r[3], sp.c[0], fma(f.r[4], sp.c[1], fma(f.r[5], sp.c[2], f.t[1])));
        const T pz = fma(f.r[6], sp.c[0], fma(f.r[7], sp.c[1], fma(f.r[8], sp.c[2], f.t[2])));
        T g[3] = {T(0), T(0), T(0)};
        T d = union_sdf<T, GRAD>(boxes, aabb, na, nb, px, py, pz, g) - sp.r;
        const bool cut = d > trunc;  // truncation_dist (src/collision.jl:84-87)
        if (cut) d = trunc;
        d -= offs;  // IneqConst: dist - margin (src/planning.jl:66)
        dmin = fmin(dmin, d);
        if (dists) st_soa(dists, sp.out, ldd, off, d);
        if (GRAD) {
            const int64_t r0 = (int64_t)sp.out * ndof;
            uint64_t zm = P.zmask;  // q columns that cannot move this chain: 0
            while (zm) {
                const int c = __builtin_ctzll(zm);
                zm &= zm - 1;
                st_soa(grads, r0 + c, ldg, off, T(0));
            }
#pragma unroll
            for (int j = 0; j < MAXA; ++j) {
                if (S[j].flags & SF_REC) {
                    T v = T(0);
                    if (j <= s_last && !cut) {
                        T jl[3];
                        if (S[j].jkind == MOT_PRISM) {
                            jl[0] = rz[j][0]; jl[1] = rz[j][1]; jl[2] = rz[j][2];
                        } else {
                            const T dx = px - ro[j][0], dy = py - ro[j][1], dz = pz - ro[j][2];
                            jl[0] = fma(rz[j][1], dz, -(rz[j][2] * dy));
                            jl[1] = fma(rz[j][2], dx, -(rz[j][0] * dz));
                            jl[2] = fma(rz[j][0], dy, -(rz[j][1] * dx));
                        }
                        v = fma(g[0], jl[0], fma(g[1], jl[1], g[2] * jl[2]));
                    }
                    uint64_t m = S[j].colmask;
                    while (m) {
                        const int c = __builtin_ctzll(m);
                        m &= m - 1;
                        st_soa(grads, r0 + c, ldg, off, v);
                    }
                }
            }
            if (P.flags & PF_BASE) {  // base columns [1 0 -y; 0 1 x; 0 0 0] (src/algorithm.jl:98-103)
                const int64_t b0 = r0 + P.n_jac;
                st_soa(grads, b0 + 0, ldg, off, cut ? T(0) : g[0]);
                st_soa(grads, b0 + 1, ldg, off, cut ? T(0) : g[1]);
                st_soa(grads, b0 + 2, ldg, off, cut ? T(0) : fma(-g[0], py - by, g[1] * (px - bx)));
            }
        }
    }
}

template <typename T, int MAXA, bool GRAD>
__global__ __launch_bounds__(256) void k_coll(const KProg<T> P, const KStep<T>* __restrict__ S,
                                              const KSphere<T>* __restrict__ sph, const KBox<T>* __restrict__ boxes,
                                              const CollArgs a, const T* __restrict__ q, int64_t ldq, int64_t n,
                                              T* __restrict__ dists, int64_t ldd, T* __restrict__ grads,
                                              int64_t ldg, T* __restrict__ min_dist) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)n) return;
    const uint32_t off = i * (uint32_t)sizeof(T);
    const bool base = (P.flags & PF_BASE) != 0;
    T bx = T(0), by = T(0), bth = T(0);
    if (base) {
        bx = ld_soa(q, P.base_col, ldq, off);
        by = ld_soa(q, P.base_col + 1, ldq, off);
        bth = ld_soa(q, P.base_col + 2, ldq, off);
    }
    T qa[MAXA];
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const int32_t c = S[s].qcol;
        qa[s] = c >= 0 ? ld_soa(q, c, ldq, off) : T(0);
    }
    Fr<T> f;
    if (base) base_frame(f, bx, by, bth);
    else set_identity(f);
    const T trunc = (T)a.truncation;
    const T offs = (T)a.offset;
    T dmin = T(INFINITY);
    T ro[MAXA][3], rz[MAXA][3];
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {  // records of unused slots are never read
        ro[s][0] = ro[s][1] = ro[s][2] = T(0);
        rz[s][0] = rz[s][1] = rz[s][2] = T(0);
    }
    const KAabb<T>* aabb = reinterpret_cast<const KAabb<T>*>(boxes + a.n_boxes);
    coll_spheres<T, MAXA, GRAD>(-1, P.sph_root0, P.sph_root1, f, P, S, sph, boxes, aabb, a.n_aabb, a.n_boxes, trunc, offs, ro,
                                rz, bx, by, off,
                          dists, ldd, grads, ldg, dmin);
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        step_a(f, S[s], qa[s], ro[s], rz[s]);
        coll_spheres<T, MAXA, GRAD>(s, S[s].sph0, S[s].sph1, f, P, S, sph, boxes, aabb, a.n_aabb, a.n_boxes, trunc,
                                    offs, ro, rz, bx, by, off,
                              dists, ldd, grads, ldg, dmin);
    }
    if (min_dist) st_soa(min_dist, 0, 0, off, dmin);
}

// --------------------------------------------------------------------------
// k_pose_residual: PoseConstraint values (src/planning.jl:125-134)
//   [t - t*; rpy(R) - rpy(R*)] with rpy = RotZYX angles (src/transform.jl:45-48)
// from the pose k_fk just wrote; elementwise over configurations.
// --------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void rpy_zyx(const T (&m)[12], T (&out)[3]) {
    // m: R11 R21 R31 R12 R22 R32 R13 R23 R33 (column-major 3x3) then t
    const T t1 = atan2_t(m[1], m[0]);
    T s1, c1;
    sincos_t(t1, &s1, &c1);
    const T t2 = atan2_t(-m[2], fma(m[1], s1, m[0] * c1));
    const T t3 = atan2_t(fma(m[6], s1, -(m[7] * c1)), fma(m[4], c1, -(m[3] * s1)));
    out[0] = t3; out[1] = t2; out[2] = t1;
}

template <typename T>
__global__ __launch_bounds__(256) void k_pose_residual(const T* __restrict__ poses, int64_t ldp,
                                                       const T* __restrict__ tgt, int64_t ldt, int64_t n, int rows,
                                                       T* __restrict__ vals, int64_t ldv) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)n) return;
    const uint32_t off = i * (uint32_t)sizeof(T);
    T a[12], b[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        a[k] = ld_soa(poses, k, ldp, off);
        b[k] = ld_soa(tgt, k, ldt, off);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) st_soa(vals, k, ldv, off, a[9 + k] - b[9 + k]);
    if (rows == 6) {
        T ra[3], rb[3];
        rpy_zyx(a, ra);
        rpy_zyx(b, rb);
#pragma unroll
        for (int k = 0; k < 3; ++k) st_soa(vals, 3 + k, ldv, off, ra[k] - rb[k]);
    }
}

inline unsigned grid_of(int64_t n, int block) { return (unsigned)((n + block - 1) / block); }

}  // namespace

// phase-A sizes compiled (the stager pads the chain to one of these: pick_chain_bound)
#define KIN_MAXA_DISPATCH(M, CALL) \
    switch (M) {                   \
    case 4: CALL(4); break;        \
    case 8: CALL(8); break;        \
    case 12: CALL(12); break;      \
    case 16: CALL(16); break;      \
    default: CALL(32); break;      \
    }

// Launches are split into chunks of kChunk configurations so that every lane
// byte offset (uint32, ld_soa / st_soa) fits in 32 bits; chunks are pointer
// offsets into the same SoA arrays (the leading dimensions do not change).
constexpr int64_t kChunk = int64_t(1) << 27;

template <typename T>
hipError_t launch_fk(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const T* q, int64_t ldq,
                     int64_t n, T* poses, int64_t ldp, T* jac, int64_t ldj, hipStream_t st) {
    for (int64_t s0 = 0; s0 < n; s0 += kChunk) {
        const int64_t c = std::min(kChunk, n - s0);
        const dim3 grid(grid_of(c, g.block)), block(g.block);
        const T* qc = q ? q + s0 : q;
        T* pc = poses ? poses + s0 : poses;
        T* jc = jac ? jac + s0 : jac;
#define KIN_FK_LAUNCH(MA) \
        hipLaunchKernelGGL((k_fk<T, MA>), grid, block, g.lds, st, P, steps, qc, ldq, c, pc, ldp, jc, ldj)
        KIN_MAXA_DISPATCH(g.maxA, KIN_FK_LAUNCH)
#undef KIN_FK_LAUNCH
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// Lanes per IK target (parallel restart attempts): enough to put ~8 waves on
// every SIMD for small batches, never more than the attempts the schedule has.
// KINHIP_IK_GROUP=<1|2|4|8> overrides (A/B).
static int ik_group(int64_t n, int n_attempts, int lanes) {
    static const int env = [] {
        const char* e = getenv("KINHIP_IK_GROUP");
        return e ? atoi(e) : 0;
    }();
    const int forced = lanes ? lanes : env;
    if (forced == 1 || forced == 2 || forced == 4 || forced == 8) return forced;
    int g = 1;
    while (g < n_attempts && g < 8 && n * g * 2 <= (int64_t(1) << 19)) g *= 2;
    return g;
}

template <typename T>
hipError_t launch_ik_dls(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const IkArgs& a,
                         const T* target, int64_t ldt, T* q, int64_t ldq, int64_t n, int32_t* iters, T* err,
                         int64_t lde, hipStream_t st) {
    const int L = a.restarts > 0 ? a.max_iters / (a.restarts + 1) : 0;
    const int natt = (L > 0 && a.max_iters > 0) ? 1 + (a.max_iters - 1) / L : 1;
    IkArgsT<T> at{a.max_iters, T(a.lambda * a.lambda), T(a.tol_pos), T(a.tol_rot), T(a.max_step), L, natt, a.seed,
                  0};
    const int G = ik_group(n, natt, a.lanes);
    const int64_t chunk = kChunk / 8;  // lane index gt = i * G stays below 2^32
    for (int64_t s0 = 0; s0 < n; s0 += chunk) {
        at.ibase = s0;
        const int64_t c = std::min(chunk, n - s0);
        const dim3 grid(grid_of(c * G, 256)), block(256);
        const T* tc = target + s0;
        T* qc = q + s0;
        int32_t* ic = iters ? iters + s0 : iters;
        T* ec = err ? err + s0 : err;
#define KIN_IK_G(MA, R, GG) \
        hipLaunchKernelGGL((k_ik_dls<T, MA, R, GG>), grid, block, 0, st, P, steps, at, tc, ldt, qc, ldq, c, ic, ec, lde)
#define KIN_IK6(MA) \
        switch (G) { case 2: KIN_IK_G(MA, 6, 2); break; case 4: KIN_IK_G(MA, 6, 4); break; \
                     case 8: KIN_IK_G(MA, 6, 8); break; default: KIN_IK_G(MA, 6, 1); }
#define KIN_IK3(MA) \
        switch (G) { case 2: KIN_IK_G(MA, 3, 2); break; case 4: KIN_IK_G(MA, 3, 4); break; \
                     case 8: KIN_IK_G(MA, 3, 8); break; default: KIN_IK_G(MA, 3, 1); }
        if (a.with_rot) {
            KIN_MAXA_DISPATCH(g.maxA, KIN_IK6)
        } else {
            KIN_MAXA_DISPATCH(g.maxA, KIN_IK3)
        }
#undef KIN_IK6
#undef KIN_IK3
#undef KIN_IK_G
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <typename T>
hipError_t launch_nakamura(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const T* pts,
                           int64_t ldpt, T* q, int64_t ldq, int64_t n, hipStream_t st) {
    for (int64_t s0 = 0; s0 < n; s0 += kChunk) {
        const int64_t c = std::min(kChunk, n - s0);
        const dim3 grid(grid_of(c, 256)), block(256);
        const T* pc = pts + s0;
        T* qc = q + s0;
#define KIN_NK_LAUNCH(MA) hipLaunchKernelGGL((k_nakamura<T, MA>), grid, block, 0, st, P, steps, pc, ldpt, qc, ldq, c)
        KIN_MAXA_DISPATCH(g.maxA, KIN_NK_LAUNCH)
#undef KIN_NK_LAUNCH
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <typename T>
hipError_t launch_coll(const KProg<T>& P, const KStep<T>* steps, const KSphere<T>* sph, const KBox<T>* boxes,
                       const LaunchGeom& g, const CollArgs& a, const T* q, int64_t ldq, int64_t n, T* dists,
                       int64_t ldd, T* grads, int64_t ldg, T* min_dist, hipStream_t st) {
    for (int64_t s0 = 0; s0 < n; s0 += kChunk) {
        const int64_t c = std::min(kChunk, n - s0);
        const dim3 grid(grid_of(c, 256)), block(256);
        const T* qc = q + s0;
        T* dc = dists ? dists + s0 : dists;
        T* gc = grads ? grads + s0 : grads;
        T* mc = min_dist ? min_dist + s0 : min_dist;
#define KIN_CO_LAUNCH(MA) \
        hipLaunchKernelGGL((k_coll<T, MA, false>), grid, block, 0, st, P, steps, sph, boxes, a, qc, ldq, c, dc, ldd, gc, ldg, mc)
#define KIN_COG_LAUNCH(MA) \
        hipLaunchKernelGGL((k_coll<T, MA, true>), grid, block, 0, st, P, steps, sph, boxes, a, qc, ldq, c, dc, ldd, gc, ldg, mc)
        if (grads) {
            KIN_MAXA_DISPATCH(g.maxA, KIN_COG_LAUNCH)
        } else {
            KIN_MAXA_DISPATCH(g.maxA, KIN_CO_LAUNCH)
        }
#undef KIN_CO_LAUNCH
#undef KIN_COG_LAUNCH
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <typename T>
hipError_t launch_pose_residual(const T* poses, int64_t ldp, const T* target, int64_t ldt, int64_t n, int rows, T* vals,
                                int64_t ldv, hipStream_t st) {
    for (int64_t s0 = 0; s0 < n; s0 += kChunk) {
        const int64_t c = std::min(kChunk, n - s0);
        hipLaunchKernelGGL((k_pose_residual<T>), dim3(grid_of(c, 256)), dim3(256), 0, st, poses + s0, ldp, target + s0,
                           ldt, c, rows, vals + s0, ldv);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

#define KIN_INSTANTIATE(T)                                                                                    \
    template hipError_t launch_fk<T>(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const T*, int64_t, \
                                     int64_t, T*, int64_t, T*, int64_t, hipStream_t);                        \
    template hipError_t launch_ik_dls<T>(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const IkArgs&, \
                                         const T*, int64_t, T*, int64_t, int64_t, int32_t*, T*, int64_t,     \
                                         hipStream_t);                                                        \
    template hipError_t launch_nakamura<T>(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const T*,    \
                                           int64_t, T*, int64_t, int64_t, hipStream_t);                      \
    template hipError_t launch_coll<T>(const KProg<T>&, const KStep<T>*, const KSphere<T>*, const KBox<T>*,   \
                                       const LaunchGeom&, const CollArgs&, const T*, int64_t, int64_t, T*,    \
                                       int64_t, T*, int64_t, T*, hipStream_t);                                \
    template hipError_t launch_pose_residual<T>(const T*, int64_t, const T*, int64_t, int64_t, int, T*, int64_t, \
                                                hipStream_t);
KIN_INSTANTIATE(float)
KIN_INSTANTIATE(double)

}  // namespace kinhip
