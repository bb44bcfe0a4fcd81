// kinhip_coll_dev.h -- device body of k_coll (swept spheres vs a union of box
// SDFs, fused with FK).  Included by kinhip_coll.hip (generic kernel) and
// embedded in the run-time specialised source (kinhip_jit.cpp).  gfx950 only.
#pragma once
#include "kinhip_device.h"

#ifndef KINHIP_COLL_FAST_TRIG
#define KINHIP_COLL_FAST_TRIG 1  // fp32: hardware sin/cos for the chain (joint_sincos, ~4e-7 abs error)
#endif

namespace kinhip {
namespace {

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
    const T mn = fmin(mx, T(0));  // 0 outside, max(q) inside (where every o is 0)
    return fma(ox, ox, fma(oy, oy, fma(oz, oz, -(mn * mn))));
}

// d from its surrogate d|d|: one square root (hardware v_sqrt_f32 for fp32, <= 1 ulp)
__device__ __forceinline__ float signed_sqrt(float k) { return copysignf(__builtin_amdgcn_sqrtf(fabsf(k)), k); }
__device__ __forceinline__ double signed_sqrt(double k) { return copysign(sqrt(fabs(k)), k); }

// KINHIP_COLL_SOFF=1 (the specialised kernels, kinhip_jit.cpp): rows addressed through soffset
// (ldo_soa / sto_soa, kinhip_device.h); the launcher runs them only within that addressing's bound
#ifndef KINHIP_COLL_SOFF
#define KINHIP_COLL_SOFF 0
#endif
#if KINHIP_COLL_SOFF
#define KIN_CO_LD ldo_soa
#define KIN_CO_ST sto_soa
#define KIN_CO_ST2 sto_soa2
#else
#define KIN_CO_LD ld_soa
#define KIN_CO_ST st_soa
#define KIN_CO_ST2 st_soa2
#endif

#ifndef KINHIP_AABB_UNROLL
#define KINHIP_AABB_UNROLL 2
#endif
// Boxes copied to LDS at kernel start (distances + gradients): the argmin box of every sphere is
// a per-lane (divergent) record, and gathering it from global memory puts a vector load behind
// the sphere's stores -- its s_waitcnt vmcnt then waits for every store the wave has issued, once
// per sphere.  An LDS gather is counted apart from the stores.  Up to kCollLdsBoxes boxes (4 KiB
// fp32); larger unions gather from global memory.
constexpr int kCollLdsBoxes = 64;

// UnionSDF of NS points at once (NS = 2: two spheres of one link share every box's data, loaded
// once through the scalar cache, and the loop overhead).  d[i] = sdf(p_i); GRAD: gw[i] = its
// analytic gradient.
// union_argmin: the surrogate minimum best[i] (and, ARG, the index bk[i] of its first box) over the
// union; box_gradient: the analytic gradient of box k at p; union_sdf = both.
template <typename T, bool ARG, int NS>
__device__ __forceinline__ void union_argmin(const KBox<T>* __restrict__ boxes, const KAabb<T>* __restrict__ aabb, int na,
                                             int nb, const T (&px)[NS], const T (&py)[NS], const T (&pz)[NS],
                                             T (&best)[NS], int (&bk)[NS]) {
    constexpr bool GRAD = ARG;
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        best[i] = T(INFINITY);
        bk[i] = 0;
    }
    // uniform loops, box data through the scalar cache; argmin keeps the first minimum (Julia's argmin)
    auto aabb_box = [&](const KAabb<T>& b, int k) {  // axis-aligned boxes: no rotation
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const T key = box_key(fabs(px[i] - b.c[0]) - b.half[0], fabs(py[i] - b.c[1]) - b.half[1],
                                  fabs(pz[i] - b.c[2]) - b.half[2]);
            if (GRAD) {
                if (key < best[i]) {
                    best[i] = key;
                    bk[i] = k;
                }
            } else {
                best[i] = fmin(best[i], key);
            }
        }
    };
    // KINHIP_AABB_UNROLL boxes per trip through one pointer that moves by whole trips, so every scalar
    // load sits at a non-negative immediate offset from it (an unroll pragma let the loop-strength
    // reduction base the pointer on the last box and rebuild each earlier address with 64-bit SALU adds)
    const KAabb<T>* __restrict__ ab = aabb;
    int k = 0;
#pragma clang loop vectorize(disable) unroll(disable)
    for (; k + KINHIP_AABB_UNROLL <= na; k += KINHIP_AABB_UNROLL, ab += KINHIP_AABB_UNROLL) {
#pragma unroll
        for (int u = 0; u < KINHIP_AABB_UNROLL; ++u) aabb_box(ab[u], k + u);
    }
#pragma clang loop vectorize(disable) unroll(disable)
    for (; k < na; ++k, ++ab) aabb_box(ab[0], k);
#pragma clang loop vectorize(disable)
    for (int k = na; k < nb; ++k) {
        const KBox<T>& b = boxes[k];
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const T qx = fabs(fma(b.inv[0], px[i], fma(b.inv[1], py[i], fma(b.inv[2], pz[i], b.inv[3])))) - b.half[0];
            const T qy = fabs(fma(b.inv[4], px[i], fma(b.inv[5], py[i], fma(b.inv[6], pz[i], b.inv[7])))) - b.half[1];
            const T qz = fabs(fma(b.inv[8], px[i], fma(b.inv[9], py[i], fma(b.inv[10], pz[i], b.inv[11])))) - b.half[2];
            const T key = box_key(qx, qy, qz);
            if (GRAD) {
                if (key < best[i]) {
                    best[i] = key;
                    bk[i] = k;
                }
            } else {
                best[i] = fmin(best[i], key);
            }
        }
    }
}

// analytic gradient of box k (a per-lane index) at p, in the box's own frame, rotated to the world
template <typename T>
__device__ __forceinline__ void box_gradient(const KBox<T>* __restrict__ boxes, const unsigned char* smem, bool use_lds,
                                             int k, T px, T py, T pz, T (&gw)[3]) {
    // explicit address spaces: the two gathers are ds_read and global_load, never one flat
    // load through a selected pointer (which the optimiser otherwise forms from the branch)
    KBox<T> b;
    if (use_lds) {
        const __attribute__((address_space(3))) KBox<T>* lb = (const __attribute__((address_space(3))) KBox<T>*)smem;
#pragma unroll
        for (int j = 0; j < 12; ++j) b.inv[j] = lb[k].inv[j];
#pragma unroll
        for (int j = 0; j < 3; ++j) b.half[j] = lb[k].half[j];
    } else {
        const __attribute__((address_space(1))) KBox<T>* gb = (const __attribute__((address_space(1))) KBox<T>*)boxes;
#pragma unroll
        for (int j = 0; j < 12; ++j) b.inv[j] = gb[k].inv[j];
#pragma unroll
        for (int j = 0; j < 3; ++j) b.half[j] = gb[k].half[j];
    }
    T l[3], q[3], gl[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        l[j] = fma(b.inv[4 * j], px, fma(b.inv[4 * j + 1], py, fma(b.inv[4 * j + 2], pz, b.inv[4 * j + 3])));
        q[j] = fabs(l[j]) - b.half[j];
    }
    const T mx = fmax(q[0], fmax(q[1], q[2]));
    if (mx > T(0)) {  // outside: d = |max(q, 0)|
        const T o[3] = {fmax(q[0], T(0)), fmax(q[1], T(0)), fmax(q[2], T(0))};
        const T oo = fma(o[0], o[0], fma(o[1], o[1], o[2] * o[2]));  // (explicit: every kernel variant rounds alike)
        T rn;  // fp32: hardware v_rsq_f32 (1 ulp) instead of the ~10-instruction IEEE division
        if constexpr (sizeof(T) == 4) rn = rsqrt_fast(oo);
        else rn = T(1) / sqrt_t(oo);
#pragma unroll
        for (int j = 0; j < 3; ++j) gl[j] = (l[j] < T(0) ? -o[j] : o[j]) * rn;
    } else {  // inside: d = max(q)
        const int im = (q[0] >= q[1] && q[0] >= q[2]) ? 0 : (q[1] >= q[2] ? 1 : 2);
#pragma unroll
        for (int j = 0; j < 3; ++j) gl[j] = (j == im) ? (l[j] < T(0) ? T(-1) : T(1)) : T(0);
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) gw[j] = fma(b.inv[j], gl[0], fma(b.inv[4 + j], gl[1], b.inv[8 + j] * gl[2]));
}

template <typename T, bool GRAD, int NS>
__device__ __forceinline__ void union_sdf(const KBox<T>* __restrict__ boxes, const KAabb<T>* __restrict__ aabb, int na,
                                          int nb, const T (&px)[NS], const T (&py)[NS], const T (&pz)[NS],
                                          T (&d)[NS], T (&gw)[NS][3], const unsigned char* smem, bool use_lds) {
    T best[NS];
    int bk[NS];
    union_argmin<T, GRAD, NS>(boxes, aabb, na, nb, px, py, pz, best, bk);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        d[i] = signed_sqrt(best[i]);
        if (GRAD) box_gradient<T>(boxes, smem, use_lds, bk[i], px[i], py[i], pz[i], gw[i]);
    }
}

// ---- boxes attached to a scene mechanism (kin_sdf_create_attached, kinhip_prog.h KSceneStep) ----
template <typename T>
struct SceneArgs {
    const KSceneGroup* groups = nullptr;
    const KSceneStep<T>* steps = nullptr;
    const T* q = nullptr;    // scene columns [cols][ld] (per sample), or one sample for the whole launch
    int64_t ld = 0;          // uniform: 1 (q[col])
    int32_t ng = 0;
    int32_t base_col = -1;   // scene planar base (x, y, theta) columns, -1: none
    int32_t uniform = 0;     // 1: every sample uses the scene column values of sample 0
};
// The group frames of a lane: in registers (12 per group), or with LF in LDS slots of the lane
// (element (g, j) at lf[(g * 12 + j) * B]: consecutive lanes, no bank conflicts) -- the specialised fp32
// door-sweep kernel, whose 2 x 12 frame registers are what keeps it at 4 waves per SIMD (KINHIP_SCENE_LDS)
template <typename T, int MAXG, bool LF = false>
struct SceneCtx {
    KSceneGroup gr[MAXG];  // the groups' descriptors, loaded once (uniform: scalar registers)
    int ng;
    T inv[LF ? 1 : MAXG][12];  // per lane: world -> group frame (row-major 3x4); MAXG >= ng (register budget)
    __attribute__((address_space(3))) T* lf = nullptr;
    int B = 0;
    __device__ __forceinline__ T at(int g, int j) const {
        if constexpr (LF) return lf[(g * 12 + j) * B];
        else return inv[g][j];
    }
    __device__ __forceinline__ void set(int g, int j, T v) {
        if constexpr (LF) lf[(g * 12 + j) * B] = v;
        else inv[g][j] = v;
    }
};
// (measured and not kept: the frames in LDS, 115 -> 103 VGPRs, still 4 waves per SIMD, door sweep 130 -> 143 us;
// with 5 waves forced, 7 VGPR spills, 144 us -- profiles/r05_scene_lds_ab.txt.  A/B build: KINHIP_SCENE_LDS=1)
#ifndef KINHIP_SCENE_LDS
#define KINHIP_SCENE_LDS 0
#endif
// whether a scene kernel of `scene_groups` groups keeps the lane frames in LDS, after the boxes (kinhip_coll.hip
// sizes the launch: 12 * scene_groups * blockDim values)
template <typename T>
__host__ __device__ constexpr bool scene_frames_in_lds(int scene_groups) {
    return KINHIP_SCENE_LDS && sizeof(T) == 4 && scene_groups > 0 && scene_groups <= 2;
}

// rotation by th about the unit axis u (Rodrigues; the reference's UnitQuaternion(cos th/2, u sin th/2)).
// fmaz / mul0: with the axis a compile-time constant (kin_plan_specialize_scene) a coordinate axis leaves
// the 2x2 block of c and s alone (the other products are structural zeros)
template <typename T>
__device__ __forceinline__ void axis_rotation(const T* __restrict__ u, T th, T (&R)[9]) {
    T s, c;
    sincos_t(th, &s, &c);
    const T v = T(1) - c, x = u[0], y = u[1], z = u[2];
    R[0] = fmaz(x * x, v, c);              R[1] = fmaz(x * y, v, -mul0(z, s)); R[2] = fmaz(x * z, v, mul0(y, s));
    R[3] = fmaz(y * x, v, mul0(z, s));     R[4] = fmaz(y * y, v, c);           R[5] = fmaz(y * z, v, -mul0(x, s));
    R[6] = fmaz(z * x, v, -mul0(y, s));    R[7] = fmaz(z * y, v, mul0(x, s));  R[8] = fmaz(z * z, v, c);
}

// the group frames of this sample (get_transform(scene, link) up to the group's moving frame), inverted
template <typename T, int MAXG, bool LF>
__device__ __forceinline__ void scene_frames(SceneCtx<T, MAXG, LF>& sc, const SceneArgs<T>& sa, uint32_t off) {
    sc.ng = sa.ng;
    const uint32_t so = sa.uniform ? 0u : off;
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
        if (g >= sa.ng) break;  // uniform
        sc.gr[g] = sa.groups[g];
        const KSceneGroup& G = sc.gr[g];
        Fr<T> f;
        if (sa.base_col >= 0)
            base_frame(f, ld_soa(sa.q, sa.base_col, sa.ld, so), ld_soa(sa.q, sa.base_col + 1, sa.ld, so),
                       ld_soa(sa.q, sa.base_col + 2, sa.ld, so));
        else
            set_identity(f);
        for (int k = G.step0; k < G.step1; ++k) {
            const KSceneStep<T>& st = sa.steps[k];
            mul_rigid(f, st.F);
            if (st.kind == MOT_REV) {
                T R[9];
                axis_rotation(st.axis, ld_soa(sa.q, st.qcol, sa.ld, so), R);
                Fr<T> h;
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int j = 0; j < 3; ++j)
                        h.r[3 * i + j] = fmaz(f.r[3 * i], R[j], fmaz(f.r[3 * i + 1], R[3 + j], mul0z(f.r[3 * i + 2], R[6 + j])));
#pragma unroll
                for (int k2 = 0; k2 < 9; ++k2) f.r[k2] = h.r[k2];
            } else if (st.kind == MOT_PRISM) {
                const T d = ld_soa(sa.q, st.qcol, sa.ld, so);
#pragma unroll
                for (int i = 0; i < 3; ++i)
                    f.t[i] = fma(fmaz(f.r[3 * i], st.axis[0], fmaz(f.r[3 * i + 1], st.axis[1], mul0z(f.r[3 * i + 2], st.axis[2]))),
                                 d, f.t[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j) sc.set(g, 4 * i + j, f.r[3 * j + i]);
            sc.set(g, 4 * i + 3, -fmaz(f.r[i], f.t[0], fmaz(f.r[3 + i], f.t[1], mul0z(f.r[6 + i], f.t[2]))));
        }
    }
}

// UnionSDF over the scene's groups: each group's boxes in its own frame (union_sdf), the first minimum
// over groups; the gradient rotated back to the world
template <typename T, bool GRAD, int NS, int MAXG, bool LF>
__device__ __forceinline__ void scene_union(const SceneCtx<T, MAXG, LF>& sc, const KBox<T>* __restrict__ boxes,
                                            const KAabb<T>* __restrict__ aabb, const T (&px)[NS], const T (&py)[NS],
                                            const T (&pz)[NS], T (&d)[NS], T (&gw)[NS][3], const unsigned char* smem,
                                            bool use_lds) {
    int wg[NS], wk[NS];  // GRAD: the winning group (-1: none) and its argmin box (index into boxes)
#pragma unroll
    for (int i = 0; i < NS; ++i) {
        d[i] = T(INFINITY);
        gw[i][0] = gw[i][1] = gw[i][2] = T(0);
        wg[i] = -1;
        wk[i] = 0;
    }
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
        if (g >= sc.ng) break;  // uniform
        const KSceneGroup& G = sc.gr[g];
        T I[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) I[j] = sc.at(g, j);
        T lx[NS], ly[NS], lz[NS];
        // Exact cull: every box of the group lies in its enclosing box (bc, bh), so the distance to that
        // box is a lower bound of the group's distance; a group that cannot come below the minimum of the
        // earlier groups (dg < d takes a group) is skipped -- with a slack beyond the rounding of both
        // distances, so the skip never changes a result.  (The door of fridge_demo.jl's scene is a small
        // group: most spheres skip it.)
        bool need = false;
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            lx[i] = fmaz(I[0], px[i], fmaz(I[1], py[i], fmaz(I[2], pz[i], I[3])));
            ly[i] = fmaz(I[4], px[i], fmaz(I[5], py[i], fmaz(I[6], pz[i], I[7])));
            lz[i] = fmaz(I[8], px[i], fmaz(I[9], py[i], fmaz(I[10], pz[i], I[11])));
            const T ox = fmax(fabs(lx[i] - (T)G.bc[0]) - (T)G.bh[0], T(0));
            const T oy = fmax(fabs(ly[i] - (T)G.bc[1]) - (T)G.bh[1], T(0));
            const T oz = fmax(fabs(lz[i] - (T)G.bc[2]) - (T)G.bh[2], T(0));
            const T lb2 = fma(ox, ox, fma(oy, oy, oz * oz));
            // d + slack (d = +inf: never culled; d < 0: only a point clearly outside the group's box)
            const T lim = fmax(d[i] + fma(fabs(d[i]), T(1e-4), T(1e-5)), T(1e-5));
            need |= !(lb2 > lim * lim);
        }
        if (!need) continue;  // (per lane: a wave skips the group when none of its lanes needs it)
        T best[NS];
        int bk[NS];
        union_argmin<T, GRAD, NS>(boxes + G.box0, aabb + G.aabb0, G.na, G.nb, lx, ly, lz, best, bk);
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            const T dg = signed_sqrt(best[i]);
            if (dg < d[i]) {
                d[i] = dg;
                if (GRAD) {
                    wg[i] = g;
                    wk[i] = G.box0 + bk[i];
                }
            }
        }
    }
    if constexpr (GRAD) {
        // the gradient once, of the winning group's argmin box (a group that does not win costs no
        // gradient): the group frame selected per lane, the box-frame point recomputed exactly as the
        // group loop formed it, and world gradient = R_g g_local, R_g = (inverse rotation)^T
#pragma unroll
        for (int i = 0; i < NS; ++i) {
            if (wg[i] < 0) continue;  // no group below +inf (NaN input): a zero gradient
            T I[12];
            if constexpr (LF) {  // the winning group's frame: one LDS read per entry at the lane's own index
#pragma unroll
                for (int j = 0; j < 12; ++j) I[j] = sc.at(wg[i], j);
            } else {
#pragma unroll
                for (int j = 0; j < 12; ++j) I[j] = sc.inv[0][j];
#pragma unroll
                for (int g = 1; g < MAXG; ++g) {
                    if (g >= sc.ng) break;  // uniform
#pragma unroll
                    for (int j = 0; j < 12; ++j) I[j] = wg[i] == g ? sc.inv[g][j] : I[j];
                }
            }
            const T lx = fmaz(I[0], px[i], fmaz(I[1], py[i], fmaz(I[2], pz[i], I[3])));
            const T ly = fmaz(I[4], px[i], fmaz(I[5], py[i], fmaz(I[6], pz[i], I[7])));
            const T lz = fmaz(I[8], px[i], fmaz(I[9], py[i], fmaz(I[10], pz[i], I[11])));
            T gg[3];
            box_gradient<T>(boxes, smem, use_lds, wk[i], lx, ly, lz, gg);
#pragma unroll
            for (int j = 0; j < 3; ++j) gw[i][j] = fmaz(I[j], gg[0], fmaz(I[4 + j], gg[1], mul0z(I[8 + j], gg[2])));
        }
    }
}

// Two spheres of a link per pass over the boxes (coll_spheres): 1 = in the min-distance kernel only
// (default), 2 = in both kernels, 0 = never.  The pair costs ~15 VGPRs: the min-distance kernel keeps
// 8 waves per SIMD and gains ~2% (fewer scalar box loads and waits); the gradient kernel would drop
// from 5 to 4 waves per SIMD and lose 5-10% (profiles/r02_coll_ab.txt).
#ifndef KINHIP_COLL_PAIRS
#define KINHIP_COLL_PAIRS 1
#endif

// Paired gradient stores (A/B knob, specialised fp32 kernels only): the two lanes of a pair swap one
// value and each writes two configurations of one row with a 64-bit store (rows c and c + 1 of a
// sphere), half the store instructions of one row per lane.  Full waves, ndof <= 16, even ld only.
#ifndef KINHIP_COLL_STPAIR
#define KINHIP_COLL_STPAIR 0
#endif
#ifndef KINHIP_JIT
#define KINHIP_JIT 0
#endif

// SCENE: 0 = a static union; else the union is attached to a scene with at most SCENE moving groups
// (the per-lane group frames take 12 registers per group, so kernels come for 2 and kMaxSceneGroups)
template <typename T, int MAXA, bool GRAD, int SCENE = 0>
__device__ __forceinline__ void coll_spheres(int s_last, int k0, int k1, const Fr<T>& f, const KProg<T>& P,
                                             const KStep<T>* __restrict__ S, const KSphere<T>* __restrict__ sph,
                                             const KBox<T>* __restrict__ boxes, const KAabb<T>* __restrict__ aabb,
                                             int na, int nb, T trunc, T offs, bool broad, const T (&bnd)[6],
                                             const T (&rm)[MAXA][3], const T (&rz)[MAXA][3], T bx, T by,
                                             uint32_t off, T* __restrict__ dists, int64_t ldd,
                                             T* __restrict__ grads, int64_t ldg, T& dmin,
                                             const unsigned char* smem, bool use_lds,
                                             const SceneCtx<T, SCENE ? SCENE : 1, scene_frames_in_lds<T>(SCENE)>* sc = nullptr) {
    const int ndof = P.n_jac + ((P.flags & PF_BASE) ? 3 : 0);
    // paired stores (KINHIP_COLL_STPAIR): every lane of the wave active, rows 8-byte aligned
    const bool pair_ok = GRAD && KINHIP_COLL_STPAIR && grads && (ldg & 1) == 0 &&
                         (((uint64_t)grads) & 7u) == 0 && __ballot(1) == ~0ull;
    // sphere centre in the world (fmz: in specialised kernels the centre is a constant, often with
    // zero components)
    auto centre = [&](const KSphere<T>& sp, T& px, T& py, T& pz) {
        px = fmz(f.r[0], sp.c[0], fmz(f.r[1], sp.c[1], fmz(f.r[2], sp.c[2], f.t[0])));
        py = fmz(f.r[3], sp.c[0], fmz(f.r[4], sp.c[1], fmz(f.r[5], sp.c[2], f.t[1])));
        pz = fmz(f.r[6], sp.c[0], fmz(f.r[7], sp.c[1], fmz(f.r[8], sp.c[2], f.t[2])));
    };
    // Broad phase (finite truncation only): every box lies inside the world-aligned box (centre
    // bnd[0..2], half extents bnd[3..5]), so a distance to it beyond trunc + r proves sdf(p) - r >
    // trunc: the reference would report the truncated value with a zero gradient, and that is
    // written without evaluating the boxes when the whole wave agrees (wave-uniform skip; the slack
    // covers rounding of the exact path).  Results are identical to evaluating every box.
    auto all_far = [&](const KSphere<T>& sp, T px, T py, T pz) -> bool {
        if (!broad) return false;
        const T ox = fmax(fabs(px - bnd[0]) - bnd[3], T(0));
        const T oy = fmax(fabs(py - bnd[1]) - bnd[4], T(0));
        const T oz = fmax(fabs(pz - bnd[2]) - bnd[5], T(0));
        const T lim = fma(trunc + sp.r, T(1.0001), T(1e-5));
        return __all(lim > T(0) && fma(ox, ox, fma(oy, oy, oz * oz)) > lim * lim);
    };
    // truncation, margin, outputs and gradient columns of one sphere (sdf value ds, gradient g)
    auto finish = [&](const KSphere<T>& sp, T px, T py, T pz, bool skipped, T ds, const T (&g)[3]) {
        T d;
        bool cut;
        if (skipped) {
            d = trunc;
            cut = true;
        } else {
            d = ds - sp.r;
            cut = d > trunc;  // truncation_dist (src/collision.jl:84-87)
            if (cut) d = trunc;
        }
        d -= offs;  // IneqConst: dist - margin (src/planning.jl:66)
        dmin = fmin(dmin, d);
        if (dists) KIN_CO_ST(dists, sp.out, ldd, off, d);
        if constexpr (GRAD && KINHIP_COLL_STPAIR && KINHIP_JIT && sizeof(T) == 4) {
            constexpr int NC = 16;
            if (ndof <= NC && pair_ok) {  // uniform
                const int64_t r0 = (int64_t)sp.out * ndof;
                T cv[NC];
#pragma unroll
                for (int c = 0; c < NC; ++c) cv[c] = T(0);  // and the columns that cannot move this chain
                const T w0 = fma(py, g[2], -(pz * g[1])), w1 = fma(pz, g[0], -(px * g[2])), w2 = fma(px, g[1], -(py * g[0]));
#pragma unroll
                for (int j = 0; j < MAXA; ++j) {
                    if (S[j].flags & SF_REC) {
                        T v = T(0);
                        if (j <= s_last && !cut) {
                            if (S[j].jkind == MOT_PRISM)
                                v = fma(g[0], rz[j][0], fma(g[1], rz[j][1], g[2] * rz[j][2]));
                            else
                                v = fma(rz[j][0], w0, fma(rz[j][1], w1, fma(rz[j][2], w2,
                                    -fma(g[0], rm[j][0], fma(g[1], rm[j][1], g[2] * rm[j][2])))));
                        }
#pragma unroll
                        for (int c = 0; c < NC; ++c)
                            if ((S[j].colmask >> c) & 1ull) cv[c] = v;
                    }
                }
                if (P.flags & PF_BASE) {
#pragma unroll
                    for (int c = 0; c < NC; ++c) {
                        if (c == P.n_jac) cv[c] = cut ? T(0) : g[0];
                        if (c == P.n_jac + 1) cv[c] = cut ? T(0) : g[1];
                        if (c == P.n_jac + 2) cv[c] = cut ? T(0) : fma(-g[0], py - by, g[1] * (px - bx));
                    }
                }
                const int par = (int)(threadIdx.x & 1u);
#pragma unroll
                for (int c = 0; c < NC; c += 2) {
                    if (c + 1 < ndof) {
                        const T send = par ? cv[c] : cv[c + 1];
                        const T recv = __shfl_xor(send, 1);
                        KIN_CO_ST2(grads, r0 + c + par, ldg, off - (uint32_t)par * 4u, par ? recv : cv[c],
                                par ? cv[c + 1] : recv);
                    } else if (c < ndof) {
                        KIN_CO_ST(grads, r0 + c, ldg, off, cv[c]);
                    }
                }
                return;
            }
        }
        if (GRAD) {
            const int64_t r0 = (int64_t)sp.out * ndof;
            uint64_t zm = P.zmask;  // q columns that cannot move this chain: 0
            while (zm) {
                const int c = __builtin_ctzll(zm);
                zm &= zm - 1;
                KIN_CO_ST(grads, r0 + c, ldg, off, T(0));
            }
            // column j = g . (z_j x (p - o_j)) = z_j . (p x g) - g . m_j with m_j = z_j x o_j
            // precomputed per configuration (k_coll), so a column costs 6 FMA instead of 12
            const T w0 = fma(py, g[2], -(pz * g[1])), w1 = fma(pz, g[0], -(px * g[2])), w2 = fma(px, g[1], -(py * g[0]));
#pragma unroll
            for (int j = 0; j < MAXA; ++j) {
                if (S[j].flags & SF_REC) {
                    T v = T(0);
                    if (j <= s_last && !cut) {
                        if (S[j].jkind == MOT_PRISM)
                            v = fma(g[0], rz[j][0], fma(g[1], rz[j][1], g[2] * rz[j][2]));
                        else
                            v = fma(rz[j][0], w0, fma(rz[j][1], w1, fma(rz[j][2], w2,
                                -fma(g[0], rm[j][0], fma(g[1], rm[j][1], g[2] * rm[j][2])))));
                    }
                    uint64_t m = S[j].colmask;
                    while (m) {
                        const int c = __builtin_ctzll(m);
                        m &= m - 1;
                        KIN_CO_ST(grads, r0 + c, ldg, off, v);
                    }
                }
            }
            if (P.flags & PF_BASE) {  // base columns [1 0 -y; 0 1 x; 0 0 0] (src/algorithm.jl:98-103)
                const int64_t b0 = r0 + P.n_jac;
                KIN_CO_ST(grads, b0 + 0, ldg, off, cut ? T(0) : g[0]);
                KIN_CO_ST(grads, b0 + 1, ldg, off, cut ? T(0) : g[1]);
                KIN_CO_ST(grads, b0 + 2, ldg, off, cut ? T(0) : fma(-g[0], py - by, g[1] * (px - bx)));
            }
        }
    };
    int k = k0;
    constexpr bool pairs = KINHIP_COLL_PAIRS == 2 || (KINHIP_COLL_PAIRS == 1 && !GRAD);
    if constexpr (pairs)
    for (; k + 1 < k1; k += 2) {  // two spheres of this link per pass over the boxes
        T px[2], py[2], pz[2], ds[2] = {T(0), T(0)}, g[2][3] = {{T(0), T(0), T(0)}, {T(0), T(0), T(0)}};
        centre(sph[k], px[0], py[0], pz[0]);
        centre(sph[k + 1], px[1], py[1], pz[1]);
        // skip only when both spheres are beyond the truncation wave-wide (the exact path gives the
        // same results for one that is)
        const bool far = all_far(sph[k], px[0], py[0], pz[0]) && all_far(sph[k + 1], px[1], py[1], pz[1]);
        if constexpr (SCENE != 0) scene_union<T, GRAD, 2, SCENE>(*sc, boxes, aabb, px, py, pz, ds, g, smem, use_lds);
        else if (!far) union_sdf<T, GRAD, 2>(boxes, aabb, na, nb, px, py, pz, ds, g, smem, use_lds);
        finish(sph[k], px[0], py[0], pz[0], far, ds[0], g[0]);
        finish(sph[k + 1], px[1], py[1], pz[1], far, ds[1], g[1]);
    }
    for (; k < k1; ++k) {
        T px[1], py[1], pz[1], ds[1] = {T(0)}, g[1][3] = {{T(0), T(0), T(0)}};
        centre(sph[k], px[0], py[0], pz[0]);
        const bool far = all_far(sph[k], px[0], py[0], pz[0]);
        if constexpr (SCENE != 0) scene_union<T, GRAD, 1, SCENE>(*sc, boxes, aabb, px, py, pz, ds, g, smem, use_lds);
        else if (!far) union_sdf<T, GRAD, 1>(boxes, aabb, na, nb, px, py, pz, ds, g, smem, use_lds);
        finish(sph[k], px[0], py[0], pz[0], far, ds[0], g[0]);
    }
}

template <typename T, int MAXA, bool GRAD, int SCENE = 0>
__device__ __forceinline__ void coll_body(const KProg<T>& P, const KStep<T>* __restrict__ S,
                                          const KSphere<T>* __restrict__ sph, const KBox<T>* __restrict__ boxes,
                                          const CollArgs& a, const T* __restrict__ q, int64_t ldq, int64_t n,
                                          T* __restrict__ dists, int64_t ldd, T* __restrict__ grads, int64_t ldg,
                                          T* __restrict__ min_dist, const Tiling& tl, unsigned char* smem,
                                          const SceneArgs<T>& sa = SceneArgs<T>{},
                                          const KAabb<T>* __restrict__ aabb_c = nullptr) {
    // gradient kernels: the union's KBox records into LDS (see kCollLdsBoxes); the launcher gives
    // the workgroup min(n_boxes, kCollLdsBoxes) * sizeof(KBox<T>) bytes
    const bool use_lds = GRAD && a.n_boxes <= kCollLdsBoxes;  // uniform
    if (use_lds) {
        const int words = a.n_boxes * (int)(sizeof(KBox<T>) / 16);
        for (int w = (int)threadIdx.x; w < words; w += (int)blockDim.x)
            reinterpret_cast<uint4*>(smem)[w] = reinterpret_cast<const uint4*>(boxes)[w];
        __syncthreads();
    }
    const uint32_t b = blockIdx.x;
    if ((uint64_t)b * blockDim.x + threadIdx.x >= (uint64_t)n) return;
    // tiled SoA (kin_coll_batch_tiled): this workgroup's tile moves the array bases (wave-uniform)
    const uint32_t t = b / tl.tile_blocks;
    q += (int64_t)t * tl.tsq;
    if (dists) dists += (int64_t)t * tl.tsp;
    if (grads) grads += (int64_t)t * tl.tsj;
    if (min_dist) min_dist += (int64_t)t * tl.tsm;
    const uint32_t i = (b - t * tl.tile_blocks) * blockDim.x + threadIdx.x;
    const uint32_t off = i * (uint32_t)sizeof(T);
    const bool base = (P.flags & PF_BASE) != 0;
    T bx = T(0), by = T(0), bth = T(0);
    if (base) {
        bx = KIN_CO_LD(q, P.base_col, ldq, off);
        by = KIN_CO_LD(q, P.base_col + 1, ldq, off);
        bth = KIN_CO_LD(q, P.base_col + 2, ldq, off);
    }
    T qa[MAXA];
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const int32_t c = S[s].qcol;
        qa[s] = c >= 0 ? KIN_CO_LD(q, c, ldq, off) : T(0);
    }
    Fr<T> f;
    if (base) base_frame(f, bx, by, bth);
    else set_identity(f);
    const T trunc = (T)a.truncation;
    const T offs = (T)a.offset;
    const bool broad = SCENE == 0 && isfinite(a.truncation);  // uniform (attached boxes: no union bound)
    constexpr bool LFS = scene_frames_in_lds<T>(SCENE);
    SceneCtx<T, SCENE ? SCENE : 1, LFS> sc;
    if constexpr (LFS) {  // this lane's frame slots after the boxes (the launcher sizes the LDS)
        const int boff = use_lds ? (a.n_boxes * (int)sizeof(KBox<T>) + 15) / 16 * 16 : 0;
        sc.lf = (__attribute__((address_space(3))) T*)((__attribute__((address_space(3))) unsigned char*)smem + boff) +
                threadIdx.x;
        sc.B = (int)blockDim.x;
    }
    if constexpr (SCENE != 0) scene_frames(sc, sa, off);  // (plain SoA only: kin_coll_batch_scene)
    const T bnd[6] = {(T)a.bc[0], (T)a.bc[1], (T)a.bc[2], (T)a.bh[0], (T)a.bh[1], (T)a.bh[2]};
    T dmin = T(INFINITY);
    T ro[MAXA][3], rz[MAXA][3];
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {  // records of unused slots are never read
        ro[s][0] = ro[s][1] = ro[s][2] = T(0);
        rz[s][0] = rz[s][1] = rz[s][2] = T(0);
    }
    // the KAabb table after the KBox array (aabb_c: a scene-specialised kernel's constant table)
    const KAabb<T>* aabb = aabb_c ? aabb_c : reinterpret_cast<const KAabb<T>*>(boxes + a.n_boxes);
    coll_spheres<T, MAXA, GRAD, SCENE>(-1, P.sph_root0, P.sph_root1, f, P, S, sph, boxes, aabb, a.n_aabb, a.n_boxes, trunc,
                                       offs, broad, bnd, ro, rz, bx, by, off, dists, ldd, grads, ldg, dmin, smem, use_lds,
                                       &sc);
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        step_a<T, KINHIP_COLL_FAST_TRIG != 0>(f, S[s], qa[s], ro[s], rz[s]);  // fp32 fast trig: see top
        if (GRAD) {  // m_s = z_s x o_s (held in ro)
            const T o0 = ro[s][0], o1 = ro[s][1], o2 = ro[s][2];
            ro[s][0] = fma(rz[s][1], o2, -(rz[s][2] * o1));
            ro[s][1] = fma(rz[s][2], o0, -(rz[s][0] * o2));
            ro[s][2] = fma(rz[s][0], o1, -(rz[s][1] * o0));
        }
        coll_spheres<T, MAXA, GRAD, SCENE>(s, S[s].sph0, S[s].sph1, f, P, S, sph, boxes, aabb, a.n_aabb, a.n_boxes,
                                           trunc, offs, broad, bnd, ro, rz, bx, by, off, dists, ldd, grads, ldg, dmin,
                                           smem, use_lds, &sc);
    }
    if (min_dist) {
        if (a.accumulate) dmin = fmin(dmin, KIN_CO_LD(min_dist, 0, 0, off));
        KIN_CO_ST(min_dist, 0, 0, off, dmin);
    }
}

}  // namespace
}  // namespace kinhip
