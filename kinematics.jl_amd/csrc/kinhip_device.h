// kinhip_device.h -- device helpers shared by the gfx950 (MI355X / CDNA4)
// kernels of the batched kinematics engine (kinhip_fk.hip, kinhip_ik.hip,
// kinhip_coll.hip).  Compiled only for --offload-arch=gfx950.
//
// Reference semantics (HiroIshida/Kinematics.jl):
//   k_fk        get_transform over many links + get_jacobian!  (src/algorithm.jl:1-106,
//               joint_transform src/mechanism.jl:90-103, rpy src/transform.jl:45-48)
//   k_ik_dls    batched damped-least-squares replacement of the SLSQP loop of
//               inverse_kinematics! (src/inverse_kinematics.jl:23-64), build-defined
//   k_nakamura  point_inverse_kinematics_nakamura (src/algorithm.jl:116-131)
//   k_coll      compute_coll_dists_and_grads! (src/collision.jl:51-94, src/sdf.jl)
//   k_pose_residual  PoseConstraint values (src/planning.jl:114-138)
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
#pragma once
#ifndef __HIPCC_RTC__  // run-time compiled sources (kinhip_jit.cpp) get only the device code
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>
#include <cstdlib>

#include <algorithm>

#include "kinhip_internal.h"
#else
#ifndef INT_MAX
#define INT_MAX 2147483647
#endif
#ifndef INFINITY
#define INFINITY __builtin_inff()
#endif
#endif
#include "kinhip_prog.h"




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
// The large-|x| path returns its results BY VALUE (in VGPRs): no pointer into the caller's private
// segment crosses the call.  Round 4 traced a MEMORY_APERTURE_VIOLATION in the generic fp64 four-lane
// collision IK to the previous form, sincos_slow(x, float* s, float* c), whose out-parameters were flat
// pointers to the caller's stack slots inside a kernel with SGPRs spilled to VGPR lanes
// (profiles/r04_ikc_fault.txt); the callee's own sincos outputs are locals, promoted to registers.
// tools/isa_check.py asserts over every product kernel that no flat access reaches private memory.
template <typename T>
struct SinCosV {
    T s, c;
};
#ifndef KINHIP_NOCALL_TRIG
#define KINHIP_NOCALL_TRIG 0  // 1 (A/B fault probe only): no out-of-line call; |x| beyond the bound -> NaN
#endif
#if KINHIP_NOCALL_TRIG
__device__ __forceinline__ SinCosV<float> sincos_slow(float) { return {__builtin_nanf(""), __builtin_nanf("")}; }
__device__ __forceinline__ SinCosV<double> sincos_slow(double) { return {__builtin_nan(""), __builtin_nan("")}; }
#else
__device__ __noinline__ SinCosV<float> sincos_slow(float x) {
    float s, c;
    sincosf(x, &s, &c);
    return {s, c};
}
__device__ __noinline__ SinCosV<double> sincos_slow(double x) {
    double s, c;
    sincos(x, &s, &c);
    return {s, c};
}
#endif

__device__ __forceinline__ void sincos_t(float x, float* s, float* c) {
    if (__builtin_expect(!(fabsf(x) < 8192.0f), 0)) {
        if (!isfinite(x)) {  // NaN / inf -> NaN, in line: no out-of-line call for a diverged lane
            *s = *c = x - x;
            return;
        }
        const SinCosV<float> r = sincos_slow(x);
        *s = r.s;
        *c = r.c;
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
        if (!isfinite(x)) {  // NaN / inf -> NaN, in line: no out-of-line call for a diverged lane
            *s = *c = x - x;
            return;
        }
        const SinCosV<double> r = sincos_slow(x);
        *s = r.s;
        *c = r.c;
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
// fp32: the hardware approximations (v_sqrt_f32 / v_rsq_f32 / v_rcp_f32, ~1 ulp) instead of
// the correctly rounded sequences; fp64: the exact operations (the oracle's arithmetic).
__device__ __forceinline__ float sqrt_fast(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ double sqrt_fast(double x) { return sqrt(x); }
__device__ __forceinline__ float rsqrt_fast(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ double rsqrt_fast(double x) { return 1.0 / sqrt(x); }
__device__ __forceinline__ float rcp_fast(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double rcp_fast(double x) { return 1.0 / x; }
// atan2(s, c) for s >= 0 (the IK rotation angle, in [0, pi]).  fp32: octant reduction to
// a = min/max in [0, 1] and atan(a) = a (1 + z P(z)), z = a^2, P a degree-6 fit
// (max abs error 1.5e-7 on [0, 1], 3.1e-7 for the angle on [0, pi], fp32; tools/atan_fit.py);
// fp64: atan2.
__device__ __forceinline__ float atan2_pos_fast(float s, float c) {
    const float ac = fabsf(c);
    const float mx = fmaxf(s, ac), mn = fminf(s, ac);
    const float a = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
    const float z = a * a;
    float p = -0.00435495f;
    p = fmaf(p, z, 0.02303899f);
    p = fmaf(p, z, -0.05777276f);
    p = fmaf(p, z, 0.0979424f);
    p = fmaf(p, z, -0.13976611f);
    p = fmaf(p, z, 0.19962715f);
    p = fmaf(p, z, -0.3333166f);
    float r = fmaf(a * z, p, a);
    r = s > ac ? 1.57079633f - r : r;
    return c < 0.0f ? 3.14159265f - r : r;
}
__device__ __forceinline__ double atan2_pos_fast(double s, double c) { return atan2(s, c); }
// atan2(y, x) over the whole plane (fp32): atan2_pos_fast's octant reduction and polynomial, the sign of y last
// (max abs error 3.1e-7; atan2(+-0, x < 0) = +-pi as the library's)
__device__ __forceinline__ float atan2_fast(float y, float x) { return copysignf(atan2_pos_fast(fabsf(y), x), y); }

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
// two consecutive configurations of one row (8 bytes at off, 8-byte aligned)
__device__ __forceinline__ void st_soa2(float* __restrict__ base, int64_t row, int64_t ld, uint32_t off, float lo, float hi) {
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(lo), __float_as_uint(hi)}, row_rsrc(base + row * ld),
                                          (int)off, 0, KINHIP_STORE_AUX);
}
__device__ __forceinline__ void st_soa(double* __restrict__ base, int64_t row, int64_t ld, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), row_rsrc(base + row * ld), (int)off, 0,
                                          KINHIP_STORE_AUX);
}

// "Narrow" SoA addressing: one buffer descriptor per array and the row folded into the
// 32-bit lane offset.  For kernels that touch many rows rarely (IK: 12 target rows, the q
// rows, 2 error rows) the per-row descriptors of ld_soa are loop-invariant, get hoisted and
// occupy 4 SGPRs each; with ~30 rows they overflow the SGPR file and spill into VGPR lanes.
// Valid while rows * ld * sizeof(T) < 2^31 (the launcher checks).
__device__ __forceinline__ float ldn_soa(const float* __restrict__ base, int64_t row, int64_t ld, uint32_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(row_rsrc(base), (int)(off + (uint32_t)(row * ld * 4)), 0, 0));
}
__device__ __forceinline__ double ldn_soa(const double* __restrict__ base, int64_t row, int64_t ld, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(row_rsrc(base),
                                                                           (int)(off + (uint32_t)(row * ld * 8)), 0, 0));
}
__device__ __forceinline__ void stn_soa(float* __restrict__ base, int64_t row, int64_t ld, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), row_rsrc(base), (int)(off + (uint32_t)(row * ld * 4)), 0,
                                          KINHIP_STORE_AUX);
}
__device__ __forceinline__ void stn_soa(double* __restrict__ base, int64_t row, int64_t ld, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), row_rsrc(base),
                                          (int)(off + (uint32_t)(row * ld * 8)), 0, KINHIP_STORE_AUX);
}

// "Row in soffset" SoA addressing: one buffer descriptor per array, the row's byte offset in the
// instruction's scalar offset (soffset) and the lane offset in the VGPR.  A row costs one scalar
// multiply-add for its offset instead of the 64-bit add plus descriptor rebuild (3 SALU) of
// ld_soa / st_soa -- the collision gradient kernel stores 126 rows per sample.  Valid while
// (rows * ld + lane span) * sizeof(T) < 2^31 (the launcher checks; kinhip_jit.cpp builds the
// specialised collision kernels with it, KINHIP_COLL_SOFF).
__device__ __forceinline__ float ldo_soa(const float* __restrict__ base, int64_t row, int64_t ld, uint32_t off) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(row_rsrc(base), (int)off, (int)(row * ld * 4), 0));
}
__device__ __forceinline__ double ldo_soa(const double* __restrict__ base, int64_t row, int64_t ld, uint32_t off) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(row_rsrc(base), (int)off, (int)(row * ld * 8), 0));
}
__device__ __forceinline__ void sto_soa(float* __restrict__ base, int64_t row, int64_t ld, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), row_rsrc(base), (int)off, (int)(row * ld * 4),
                                          KINHIP_STORE_AUX);
}
__device__ __forceinline__ void sto_soa2(float* __restrict__ base, int64_t row, int64_t ld, uint32_t off, float lo,
                                         float hi) {
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(lo), __float_as_uint(hi)}, row_rsrc(base), (int)off,
                                          (int)(row * ld * 4), KINHIP_STORE_AUX);
}
__device__ __forceinline__ void sto_soa(double* __restrict__ base, int64_t row, int64_t ld, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), row_rsrc(base), (int)off, (int)(row * ld * 8),
                                          KINHIP_STORE_AUX);
}

template <typename T>
__device__ __forceinline__ void set_identity(Fr<T>& f) {
#pragma unroll
    for (int k = 0; k < 9; ++k) f.r[k] = (k % 4 == 0) ? T(1) : T(0);
    f.t[0] = f.t[1] = f.t[2] = T(0);
}

// Products with a coefficient of the staged program.  In the generic kernels
// the coefficient is a run-time (uniform) value and these are plain fma/mul.
// In plan-specialised kernels (kinhip_jit.cpp) it is a compile-time constant:
// a term with an exactly-zero coefficient is dropped and `acc + 0` is not
// formed, which the IEEE rules would otherwise keep (x * 0 is NaN for x = inf,
// x + 0 flips -0).  For finite inputs the result equals the generic one (up to
// the sign of a zero).
template <typename T>
__device__ __forceinline__ T fmz(T a, T F, T acc) {
    if (__builtin_constant_p(F) && F == T(0)) return acc;
    if (__builtin_constant_p(acc) && acc == T(0)) return a * F;
    return fma(a, F, acc);
}
template <typename T>
__device__ __forceinline__ T mulz(T a, T F) {
    if (__builtin_constant_p(F) && F == T(0)) return T(0);
    return a * F;
}

// acc - a * b with the term dropped when a or b is a compile-time zero, and a * b = 0 when a is one: the
// structural zeros of a specialised kernel's normal equations (variables that share no row, e.g. the two
// arms of a two-arm robot) then cost no instruction in its factorisation.  Equal to fma(-a, b, acc) /
// a * b for finite operands (up to the sign of a zero), so specialised and generic kernels agree.
template <typename T>
__device__ __forceinline__ T fnz(T a, T b, T acc) {
    if ((__builtin_constant_p(a) && a == T(0)) || (__builtin_constant_p(b) && b == T(0))) return acc;
    return fma(-a, b, acc);
}
template <typename T>
__device__ __forceinline__ T mul0(T a, T b) {
    if (__builtin_constant_p(a) && a == T(0)) return T(0);
    return a * b;
}
// acc + a * b with the term dropped when a or b is a compile-time zero: the scene tables of a
// scene-specialised collision kernel (kin_plan_specialize_scene) fold a planar base's and a fixed-axis
// joint's structural zeros out of the per-lane group frames.  fma(a, b, acc) otherwise.
template <typename T>
__device__ __forceinline__ T fmaz(T a, T b, T acc) {
    if ((__builtin_constant_p(a) && a == T(0)) || (__builtin_constant_p(b) && b == T(0))) return acc;
    return fma(a, b, acc);
}
template <typename T>
__device__ __forceinline__ T mul0z(T a, T b) {
    if ((__builtin_constant_p(a) && a == T(0)) || (__builtin_constant_p(b) && b == T(0))) return T(0);
    return a * b;
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
        g.r[3 * i + 0] = fmz(a, F0, fmz(b, F4, mulz(c, F8)));
        g.r[3 * i + 1] = fmz(a, F1, fmz(b, F5, mulz(c, F9)));
        g.r[3 * i + 2] = fmz(a, F2, fmz(b, F6, mulz(c, F10)));
        g.t[i] = fmz(a, F3, fmz(b, F7, fmz(c, F11, f.t[i])));
    }
    f = g;
}

template <typename T>
__device__ __forceinline__ void mul_rigid_regs(Fr<T>& out, const Fr<T>& f, const T (&F)[12]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const T a = f.r[3 * i], b = f.r[3 * i + 1], c = f.r[3 * i + 2];
        out.r[3 * i + 0] = fmz(a, F[0], fmz(b, F[4], mulz(c, F[8])));
        out.r[3 * i + 1] = fmz(a, F[1], fmz(b, F[5], mulz(c, F[9])));
        out.r[3 * i + 2] = fmz(a, F[2], fmz(b, F[6], mulz(c, F[10])));
        out.t[i] = fmz(a, F[3], fmz(b, F[7], fmz(c, F[11], f.t[i])));
    }
}

// joint motion in the canonical frame (axis = local z), branch-free in the
// joint kind: revolute -> (c, s, 0), prismatic -> (1, 0, scale*q), none -> (1, 0, 0)
// Trig for the joint angle.  FT (fast trig, fp32 IK only): the hardware v_sin_f32 / v_cos_f32
// (max abs error 3.6e-7 over [-3.5, 3.5], tools/sin_probe.hip) instead of the ~20-instruction
// reduction + polynomial -- inside an iterative solver checked against a 1e-3 tolerance.
template <bool FT, typename T>
__device__ __forceinline__ void joint_sincos(T th, T* s, T* c) {
    if constexpr (FT && sizeof(T) == 4) {
        const float r = th * 0.15915494309189535f;  // the hardware ops take revolutions
        *s = __builtin_amdgcn_sinf(r);
        *c = __builtin_amdgcn_cosf(r);
    } else {
        sincos_t(th, s, c);
    }
}

template <typename T, bool FT = false>
__device__ __forceinline__ void motion(Fr<T>& f, int32_t kind, int32_t flags, T scale, T qv) {
    if (__builtin_constant_p(kind) && __builtin_constant_p(flags)) {  // specialised plan: kind known
        if (kind == MOT_REV) {
            T th = qv;
            if (flags & SF_SCALE) {
                T sh, ch;
                sincos_t(T(0.5) * qv, &sh, &ch);
                th = T(2) * atan2_t(scale * sh, ch);
            }
            T s, c;
            joint_sincos<FT>(th, &s, &c);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const T a = f.r[3 * i], b = f.r[3 * i + 1];
                f.r[3 * i] = fma(a, c, b * s);
                f.r[3 * i + 1] = fma(b, c, -(a * s));
            }
        } else if (kind == MOT_PRISM) {
            const T d = scale * qv;
#pragma unroll
            for (int i = 0; i < 3; ++i) f.t[i] = fma(f.r[3 * i + 2], d, f.t[i]);
        }
        return;
    }
    // generic: branch-free in the kind (a uniform branch per step splits the
    // unrolled chain into blocks and costs more than it saves, profiles/r01_fk_branch_ab.txt)
    const bool rev = kind == MOT_REV;
    T th = rev ? qv : T(0);
    if (flags & SF_SCALE) {  // UnitQuaternion normalisation of a non-unit axis
        T sh, ch;
        sincos_t(T(0.5) * qv, &sh, &ch);
        th = T(2) * atan2_t(scale * sh, ch);
    }
    T s, c;
    joint_sincos<FT>(th, &s, &c);
    const T d = (kind == MOT_PRISM) ? scale * qv : T(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const T a = f.r[3 * i], b = f.r[3 * i + 1];
        f.r[3 * i] = fma(a, c, b * s);
        f.r[3 * i + 1] = fma(b, c, -(a * s));
        f.t[i] = fma(f.r[3 * i + 2], d, f.t[i]);
    }
}

// rpy(tf) (src/transform.jl:45-48: RotZYX angles as [roll, pitch, yaw]) of a row-major rotation,
// and the rpy_derivative! coefficients at it (src/algorithm.jl:56-63, a = -rpy):
//   d(rpy)/dt = [k0 x + k1 y, k2 x + k3 y, k4 x + k5 y + z] for an angular velocity (x, y, z)
// FAST (the fp32 IK kernels, KINHIP_IK_FAST_ATAN): the polynomial atan2 (atan2_fast, 3.1e-7 abs), the hardware
// sin / cos (3.6e-7 abs) and v_rcp_f32 in place of atan2f, the reduced sincos and the IEEE division -- inside an
// iterative solve whose residual is checked against tol_rot (the fp64 kernels keep the exact functions).
template <bool FAST = false, typename T>
__device__ __forceinline__ void rpy_and_rate(const T (&r)[9], T (&rpy)[3], T (&k)[6]) {
    constexpr bool F = FAST && sizeof(T) == 4;
    auto at2 = [](T y, T x) -> T {
        if constexpr (F) return atan2_fast(y, x);
        else return atan2_t(y, x);
    };
    const T t1 = at2(r[3], r[0]);
    T s1, c1;
    joint_sincos<F>(t1, &s1, &c1);
    const T t2 = at2(-r[6], fma(r[3], s1, r[0] * c1));
    const T t3 = at2(fma(r[2], s1, -(r[5] * c1)), fma(r[4], c1, -(r[1] * s1)));
    rpy[0] = t3; rpy[1] = t2; rpy[2] = t1;
    T s2, c2;
    joint_sincos<F>(t2, &s2, &c2);  // a2 = -t2: cos(a2) = c2, sin(a2) = -s2; a3 = -t1: cos = c1, sin = -s1
    T ic2;
    if constexpr (F) ic2 = rcp_fast(c2);
    else ic2 = T(1) / c2;
    k[0] = c1 * ic2; k[1] = s1 * ic2;
    k[2] = -s1; k[3] = c1;
    k[4] = c1 * s2 * ic2; k[5] = s1 * s2 * ic2;
}

// angle difference wrapped to (-pi, pi]
template <typename T>
__device__ __forceinline__ T wrap_pi(T d) {
    const T tp = T(6.283185307179586476925286766559);
    return d - tp * rint(d * T(0.15915494309189533576888376337251));
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
// profiles/r01_store_probe.txt.  Round 4 again, with the occupancy cap: the
// staged pattern probe 3-9% slower than this one, a staged k_fk 4x slower --
// profiles/r04_fk_staged_stores_ab.txt; not kept.)
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
template <typename T, bool FT = false>
__device__ __forceinline__ void step_a(Fr<T>& f, const KStep<T>& st, T qv, T (&o)[3], T (&z)[3]) {
    mul_rigid(f, st.F);
    o[0] = f.t[0]; o[1] = f.t[1]; o[2] = f.t[2];  // _get_joint_axis, src/algorithm.jl:42-54
    const T sc = st.scale;
    z[0] = f.r[2] * sc; z[1] = f.r[5] * sc; z[2] = f.r[8] * sc;
    motion<T, FT>(f, st.kind, st.flags, sc, qv);
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


}  // namespace kinhip
