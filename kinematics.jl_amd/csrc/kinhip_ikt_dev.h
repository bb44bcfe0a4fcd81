// kinhip_ikt_dev.h -- device body of k_ik_tree: batched collision-aware IK, the second stage of
// inverse_kinematics!(m, link, joints, target, sscc, sdf; use_bistage) (src/inverse_kinematics.jl:
// 1-21): the pose objective subject to IneqConst(sscc, joints, sdf, 1, margin) (src/planning.jl:55-68,
// every swept sphere at least `margin` from the UnionSDF).  Included by kinhip_ik.hip (generic
// kernels) and embedded in the run-time specialised source (kinhip_jit.cpp).  gfx950 only.
//
// The program (KIkcProg / KIkcStep, kinhip_prog.h) is the needed kinematic tree: spheres may hang off
// any moving chain (both arms of a two-arm robot, head / torso links), the target link off another;
// the variables are the q columns (+ the planar base), each moved by one joint of the tree.  The
// boxes may be a static UnionSDF or one attached to a scene mechanism (kin_sdf_create_attached) whose
// joint values are given per target (a door angle per target: fridge_demo.jl).
#pragma once
#include "kinhip_coll_dev.h"
#include "kinhip_ik_dev.h"

// Contraction only inside one expression (a * b + c): the specialised kernels fold constants into the
// instruction stream, and fusing across statements would then differ from the generic kernels
#ifndef KINHIP_CONTRACT_FAST
#define KINHIP_CONTRACT_FAST 0
#endif
#if KINHIP_CONTRACT_FAST
#pragma clang fp contract(fast)
#else
#pragma clang fp contract(on)
#endif

// the specialised kernels unroll the tree walk and the sphere loops (constant trip counts)
#ifdef KINHIP_JIT
#define KIN_IKT_UNROLL _Pragma("unroll")
#else
#define KIN_IKT_UNROLL
#endif

// Diagnostic section stamps (tools only: KINHIP_JIT_DEFS=-DKINHIP_IKT_SECT=<k> in the A/B build,
// tools/ikt_sect.py): the cycles of iteration section k (1 tree walk, 2 sphere distances + rows, 3 rows into
// the normal equations, 4 pose error + checks, 5 pose rows, 6 factorisation + solves, 7 step + loop top)
// summed over the writer lane's iterations replace err row 0, its cycles from the first iteration to the
// write err row 1.  Never in a product build.
#ifndef KINHIP_IKT_SECT
#define KINHIP_IKT_SECT 0
#endif
#if KINHIP_IKT_SECT
#define KIN_IKT_STAMP(k)                                                   \
    do {                                                                   \
        uint64_t t_;                                                       \
        __builtin_amdgcn_sched_barrier(0);                                 \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                 \
        if ((k) == KINHIP_IKT_SECT) sect_acc += t_ - sect_prev;            \
        sect_prev = t_;                                                    \
        if (sect_t0 == 0) sect_t0 = t_;                                    \
    } while (0)
#else
#define KIN_IKT_STAMP(k) \
    do {                 \
    } while (0)
#endif

namespace kinhip {
namespace {

// Constraint handling of the collision-aware IK (kin_ik_coll_params)
template <typename T>
struct IkcArgsT {
    T margin;  // IneqConst margin (the reference's stage 2 uses 0.02)
    T band;    // a sphere with d < margin + band is pushed towards margin + band
    T weight;  // weight of a sphere's row against the pose rows
    T feas;    // converged only when every sphere has d >= margin - feas
};

// a[i] for a uniform (generic kernel) or constant (specialised kernel) index: selects, never a
// dynamically indexed register array (which the compiler would move to scratch memory)
template <typename T, int N>
__device__ __forceinline__ T pick(const T (&a)[N], int i) {
    T v = a[0];
#pragma unroll
    for (int k = 1; k < N; ++k) v = (i == k) ? a[k] : v;
    return v;
}
// a[i] for a per-lane (divergent) index: a binary tree of selects on the bits of i.  (pick's chain of
// `i == k` selects is recognised as a dynamic vector index, which a divergent index lowers through scratch
// memory: a store of the whole array and an indexed load per use.)  Indices >= N give a[N - 1].
template <typename T, int N>
__device__ __forceinline__ T pick_lane(const T (&a)[N], int i) {
    constexpr int B = N <= 1 ? 0 : N <= 2 ? 1 : N <= 4 ? 2 : N <= 8 ? 3 : N <= 16 ? 4 : 5;
    T t[1 << B];
#pragma unroll
    for (int k = 0; k < (1 << B); ++k) t[k] = a[k < N ? k : N - 1];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const bool bit = (i >> b) & 1;
#pragma unroll
        for (int k = 0; k < (1 << (B - 1 - b)); ++k) t[k] = bit ? t[2 * k + 1] : t[2 * k];
    }
    return t[0];
}
template <int V>
struct IntC {
    static constexpr int value = V;
};
// a[O + i] for a per-lane i in [0, S) (a lane's row of the O-th round of S rows; O + i >= N gives a[N - 1])
template <int O, int S, typename T, int N>
__device__ __forceinline__ T pick_round(const T (&a)[N], int i) {
    constexpr int M = N - O < S ? N - O : S;  // rows of this round that exist
    T sub[M > 0 ? M : 1];
#pragma unroll
    for (int k = 0; k < (M > 0 ? M : 1); ++k) sub[k] = a[M > 0 ? O + k : N - 1];
    return pick_lane(sub, i);
}
template <typename T, int N>
__device__ __forceinline__ void put(T (&a)[N], int i, T v) {
#pragma unroll
    for (int k = 0; k < N; ++k) a[k] = (i == k) ? v : a[k];
}
template <typename T, int N>
__device__ __forceinline__ void pick_frame(Fr<T>& f, const Fr<T> (&a)[N], int i) {
#pragma unroll
    for (int k = 0; k < N; ++k)
        if (i == k) f = a[k];
}
template <typename T, int N>
__device__ __forceinline__ void put_frame(Fr<T> (&a)[N], int i, const Fr<T>& f) {
#pragma unroll
    for (int k = 0; k < N; ++k)
        if (i == k) a[k] = f;
}

// The IneqConst row of one sphere (k_coll's gradient, src/collision.jl:67-94): a_v = g . d(c)/d(q_v) for
// the variables moving the sphere's frame (anc), 0 elsewhere.  Joints: revolute z_v . (c x g) - g . m_v
// (m = z x o, the record), prismatic g . z_v; base [g0, g1, -g0 (c_y - b_y) + g1 (c_x - b_x)].
template <typename T, int MAXV>
__device__ __forceinline__ void sphere_row(const KIkcProg<T>& P, uint32_t anc, T px, T py, T pz, const T (&g)[3],
                                           const T (&rz)[MAXV][3], const T (&rm)[MAXV][3], const T (&b)[3],
                                           T (&av)[MAXV]) {
    const T w0 = fma(py, g[2], -(pz * g[1]));
    const T w1 = fma(pz, g[0], -(px * g[2]));
    const T w3 = fma(px, g[1], -(py * g[0]));
    const bool base = P.base_col >= 0;  // (base_col = -1 without a base: no variable is a base column)
#pragma unroll
    for (int v = 0; v < MAXV; ++v) {
        T x;
        if (base && v == P.base_col) x = g[0];
        else if (base && v == P.base_col + 1) x = g[1];
        else if (base && v == P.base_col + 2) x = fma(-g[0], py - b[1], g[1] * (px - b[0]));
        else if ((P.prism_mask >> v) & 1u) x = fma(g[0], rz[v][0], fma(g[1], rz[v][1], g[2] * rz[v][2]));
        else
            x = fma(rz[v][0], w0, fma(rz[v][1], w1, fma(rz[v][2], w3,
                    -fma(g[0], rm[v][0], fma(g[1], rm[v][1], g[2] * rm[v][2])))));
        av[v] = ((anc >> v) & 1u) ? x : T(0);
    }
}

// w^2 a a^T and w^2 viol a into the lower triangle of the normal equations, over the variables of anc
// A[r][c] = fma(w[r], x[c], A[r][c]) for every r, c <= r of `mask` (the lower triangle's entries that row r
// and column c both reach; others untouched).  fp32 with KINHIP_IKT_PK: entries (r, c) and (r, c + 1) of one
// row as one v_pk_fma_f32 with w[r] broadcast where both are in the mask -- each element the same fma, so the
// results are identical (one wave per SIMD issues a packed FMA in ~1.5x the time of a scalar one,
// tools/pk_probe.hip: the pair costs 0.75 of its scalar FMAs)
#ifndef KINHIP_IKT_PK
#define KINHIP_IKT_PK 1
#endif
template <typename T, int MAXV>
__device__ __forceinline__ void lower_rank1(T (&A)[MAXV][MAXV], const T (&w)[MAXV], const T (&x)[MAXV], uint32_t mask) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    // (the pairs only where the mask is a constant -- the specialised kernels; the generic ones keep the
    // scalar loop rather than a run-time test per pair)
    if (!__builtin_constant_p(mask)) {
#pragma unroll
        for (int r = 0; r < MAXV; ++r) {
            if (!((mask >> r) & 1u)) continue;
#pragma unroll
            for (int c = 0; c <= r; ++c)
                if ((mask >> c) & 1u) A[r][c] = fma(w[r], x[c], A[r][c]);
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < MAXV; ++r) {
        if (!((mask >> r) & 1u)) continue;
#pragma unroll
        for (int c = 0; c <= r; ++c) {
            if (!((mask >> c) & 1u)) continue;
            if constexpr (KINHIP_IKT_PK && sizeof(T) == 4) {
                if (c + 1 <= r && ((mask >> (c + 1)) & 1u) && (c & 1) == 0) {
                    const f2 v = __builtin_elementwise_fma(f2{(float)w[r], (float)w[r]}, f2{(float)x[c], (float)x[c + 1]},
                                                           f2{(float)A[r][c], (float)A[r][c + 1]});
                    A[r][c] = (T)v.x;
                    A[r][c + 1] = (T)v.y;
                    continue;
                }
                if (c >= 1 && (c & 1) == 1 && ((mask >> (c - 1)) & 1u)) continue;  // (done with its pair)
            }
            A[r][c] = fma(w[r], x[c], A[r][c]);
        }
    }
}

template <typename T, int MAXV>
__device__ __forceinline__ void accum_row(T (&A)[MAXV][MAXV], T (&bv)[MAXV], const T (&av)[MAXV], T viol, T w2,
                                          uint32_t anc) {
    T wr[MAXV];
#pragma unroll
    for (int r = 0; r < MAXV; ++r) {
        wr[r] = w2 * av[r];
        if ((anc >> r) & 1u) bv[r] = fma(wr[r], viol, bv[r]);
    }
    lower_rank1<T, MAXV>(A, wr, av, anc);
}

// min over the S lanes of an aligned group (S <= 16, inside one DPP row): quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror -- every lane ends with the same value
template <int S>
__device__ __forceinline__ float row_group_min(float v) {
    if constexpr (S >= 2) v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)));
    if constexpr (S >= 4) v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false)));
    if constexpr (S >= 8) v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false)));
    if constexpr (S >= 16) v = fminf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false)));
    return v;
}
template <int CTL>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
template <int S>
__device__ __forceinline__ double row_group_min(double v) {
    if constexpr (S >= 2) v = fmin(v, dpp_f64<0xB1>(v));
    if constexpr (S >= 4) v = fmin(v, dpp_f64<0x4E>(v));
    if constexpr (S >= 8) v = fmin(v, dpp_f64<0x141>(v));
    if constexpr (S >= 16) v = fmin(v, dpp_f64<0x140>(v));
    return v;
}

// value of lane `src` (inside the caller's lane group) for every lane of the group: ds_bpermute
__device__ __forceinline__ float lane_bcast(float v, int src) { return __int_as_float(__shfl(__float_as_int(v), src)); }
__device__ __forceinline__ double lane_bcast(double v, int src) { return __shfl(v, src); }

// value of lane l of each 16-lane DPP row for every lane of that row (v_mov_b32_dpp row_newbcast:l, a VALU
// move instead of an LDS round trip); l must fold to a constant (the specialised kernels' unrolled loops)
template <int CTL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTL, 0xF, 0xF, false));
}
template <typename T>
__device__ __forceinline__ T row_bcast16(T v, int l) {
#define KIN_RB(n) \
    case n:       \
        if constexpr (sizeof(T) == 4) return dpp_f32<0x150 + n>(v); else return dpp_f64<0x150 + n>(v);
    switch (l) {
        KIN_RB(0) KIN_RB(1) KIN_RB(2) KIN_RB(3) KIN_RB(4) KIN_RB(5) KIN_RB(6) KIN_RB(7)
        KIN_RB(8) KIN_RB(9) KIN_RB(10) KIN_RB(11) KIN_RB(12) KIN_RB(13) KIN_RB(14)
        default: if constexpr (sizeof(T) == 4) return dpp_f32<0x15F>(v); else return dpp_f64<0x15F>(v);
    }
#undef KIN_RB
}

// min over the G attempt groups of a target (lanes S apart; v uniform inside each group): DPP inside a quad
// for S = 1; a target that fills the wave (G * S = 64) reads each group's value with v_readlane and takes the
// minimum in scalar registers (no LDS round trip: two dependent ds_bpermute sat on the one-wave critical path
// of every iteration); else ds_bpermute
template <int G, int S>
__device__ __forceinline__ int attempt_min(int v) {
    if constexpr (S == 1) {
        return group_min<G>(v);
    } else if constexpr (G * S == 64) {
        int m = __builtin_amdgcn_readlane(v, 0);
#pragma unroll
        for (int g = 1; g < G; ++g) m = min(m, __builtin_amdgcn_readlane(v, g * S));
        return m;
    } else {
#pragma unroll
        for (int w = S; w < G * S; w <<= 1) v = min(v, __shfl_xor(v, w));
        return v;
    }
}
template <int G, int S, typename T>
__device__ __forceinline__ T attempt_min_t(T v) {
    if constexpr (G * S == 64 && S > 1 && sizeof(T) == 4) {
        float m = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
#pragma unroll
        for (int g = 1; g < G; ++g) m = fminf(m, __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), g * S)));
        return m;
    } else {
#pragma unroll
        for (int w = S; w < G * S; w <<= 1) v = fmin(v, __shfl_xor(v, w));
        return v;
    }
}

// starting angles of an attempt: attempt 0 from q0; attempt k >= 1 re-draws every free joint variable
// within its limits (U[-pi, pi] if unbounded) from the counter hash of k_ik_dls (ik_seed_u01), other
// variables from q0 (the base: the caller).  With a second start pose (a.q_alt, kin_ik_coll_batch_alt) attempt 1
// takes its free joint variables from q_alt instead of a draw (and every restart its base from q_alt).
template <typename T, int MAXV>
__device__ __forceinline__ void ikt_start(const KIkcProg<T>& P, const IkArgsT<T>& a, const T* __restrict__ q,
                                          int64_t ldq, uint32_t off, int64_t gi, int att, T (&qs)[MAXV]) {
#pragma unroll
    for (int v = 0; v < MAXV; ++v) {
        if (v >= P.n_q) {
            qs[v] = T(0);
            continue;
        }
        if (att == 1 && a.q_alt && ((P.free_mask & P.joint_mask) >> v) & 1u) {
            qs[v] = ld_soa(a.q_alt, v, ldq, off);
        } else if (att > 0 && ((P.free_mask & P.joint_mask) >> v) & 1u) {
            double lo = (double)P.vlo[v], hi = (double)P.vhi[v];
            if (!isfinite(lo) || !isfinite(hi)) { lo = -3.14159265358979323846; hi = 3.14159265358979323846; }
            qs[v] = (T)(lo + (hi - lo) * ik_seed_u01(a.seed, gi, att, v));
        } else {
            qs[v] = ld_soa(q, v, ldq, off);
        }
    }
}

// k_ik_tree.  Lanes: G attempt groups of S lanes per target (G * S <= 64, aligned).  Lane group `ga`
// of a target runs attempts ga, ga + G, ... of k_ik_dls's restart schedule; a group stops once a
// lower attempt of its target has converged.  The S lanes of a group evaluate the same iteration:
// every lane walks the tree (the chain is short), the spheres are shared out (lane j takes spheres j,
// j + S, ...: its sphere's UnionSDF distance, analytic gradient and IneqConst row), and the sphere
// rows enter the normal equations in sphere order, broadcast from their lane -- the same operations
// in the same order as one lane doing every sphere (S = 1), so the results are identical for every
// S and G.  Per iteration ONE damped Gauss-Newton step on the normal equations over the free
// variables:
//     (J^T J + w^2 sum_k a_k^T a_k + lambda^2 I) dq = J^T e + w^2 sum_k a_k^T (margin + band - d_k)
// over the spheres with d_k < margin + band (a one-sided penalty: it pushes only while a sphere is
// too close, so in the null space of the pose task the arm moves out to the band while the pose
// error goes to zero); converged when |dp| < tol_pos, |rot| < tol_rot and every d_k >= margin - feas.
// Joint limits: a joint on a limit pushed further out (by this step if it was free, by the right-hand
// side if it was held) is held out of the next step; q is clamped to the limits.  Output: the lowest
// converged attempt, else the attempt whose end state has the lowest merit
// |dp|^2 + |rot|^2 + w^2 max(0, margin - min_k d_k)^2 (ties: the lower attempt) -- NLopt likewise
// returns the best point it found.  NR: rounds of spheres per lane (ceil(n_sph / S); S > 1 only in
// the specialised kernels, where the program is constant).  MAXG > 0: boxes attached to a scene,
// one set of scene joint values per target (sa).
// S > 1: the rows of the normal equations formed by every lane of the group (0) or owned by the group's lanes
// and gathered (1; A/B: KINHIP_JIT_DEFS=-DKINHIP_IKT_OWN=1) -- identical results.  Ownership cuts the loop's
// FMAs 1,140 -> 658 (offline ISA) and yet measured slower on every leg (stage 2 of f3 0.152 -> 0.231 ms, the
// scene door 0.198 -> 0.349, PR2 0.67 -> 2.29; profiles/r05_ikt_own_ab.txt): not kept
#ifndef KINHIP_IKT_OWN
#define KINHIP_IKT_OWN 0
#endif
// S > 1 (default): the normal equations distributed over the group's lanes through LDS.  Each sphere lane
// stores its rows (w^2 a, a, viol), every lane the pose rows J (and e); lane sl then forms the entries sl,
// sl + S, ... of the system -- entry (r, c) = sum over the in-band spheres, in sphere order, of
// fma(w^2 a_k[r], a_k[c], .), then over the pose rows, in row order, of fma(J[i][r], J[i][c], .); the
// right-hand side is column MAXV (a_k[MAXV] = viol_k, J[i][MAXV] = e_i) -- the same FMAs in the same order as
// the one-lane kernel, so the results stay identical for every S -- and the group reads the assembled system
// back for the (replicated) factorisation.  The replicated form broadcast every in-band sphere row by DPP and
// had every lane form every entry: ~50 instructions per in-band sphere and ~300 for the pose rows on the
// one-wave critical path of the batch's slowest target (offline ISA of the f3 kernel).  The masks of the
// one-lane form (a sphere's variables, the target's) are left out: a row is 0 outside them, and fma(0, x, s)
// = s for the finite, never negative-zero sums here.  0: the replicated form (A/B build).
#ifndef KINHIP_IKT_LDSNE
#define KINHIP_IKT_LDSNE 1
#endif
// LDS layout of one attempt group's system (elements of T): NSR sphere rows [w^2 a (MAXV), a (MAXV), viol]
// padded to RW, ROWS pose rows [J (MAXV), e] padded to JW, then the NE assembled entries (row r: c = 0..r, rhs)
template <int MAXV, int ROWS, int NSR>
struct IktNe {
    static constexpr int RW = (2 * MAXV + 1 + 3) & ~3;
    static constexpr int JW = (MAXV + 1 + 3) & ~3;
    static constexpr int NE = MAXV * (MAXV + 3) / 2;
    static constexpr int JB = NSR * RW;
    static constexpr int NB = JB + ROWS * JW;
    static constexpr int SIZE = (NB + NE + 3) & ~3;
    static constexpr int st(int r) { return r * (r + 3) / 2; }  // first entry of row r
};
template <typename T, int N>
__device__ __forceinline__ T* ikt_ne_lds() {
    __shared__ __attribute__((aligned(16))) T buf[N];
    return buf;
}
template <typename T, int MAXV, int ROWS, int G, int S, int NR, int MAXG>
__device__ __forceinline__ void ikt_body(const KIkcProg<T>& P, const KIkcStep<T>* __restrict__ St,
                                         const KSphere<T>* __restrict__ sph, const KBox<T>* __restrict__ boxes,
                                         const CollArgs& ca, const IkcArgsT<T>& cz, const IkArgsT<T>& a,
                                         const SceneArgs<T>& sa, const T* __restrict__ tgt, int64_t ldt,
                                         T* __restrict__ q, int64_t ldq, int64_t n, int32_t* __restrict__ iters,
                                         T* __restrict__ err, int64_t lde, unsigned char* smem) {
    static_assert(G == 1 || G == 2 || G == 4 || G == 8, "attempt groups");
    static_assert(S == 1 || S == 2 || S == 4 || S == 8 || S == 16, "sphere lanes inside a DPP row");
    static_assert(G * S <= 64 && MAXV <= kIkcMaxVars, "lane groups inside a wave");
    const bool use_lds = ca.n_boxes <= kCollLdsBoxes;  // argmin box gathers from LDS (k_coll)
    if (use_lds) {
        const int words = ca.n_boxes * (int)(sizeof(KBox<T>) / 16);
        for (int w = (int)threadIdx.x; w < words; w += (int)blockDim.x)
            reinterpret_cast<uint4*>(smem)[w] = reinterpret_cast<const uint4*>(boxes)[w];
        __syncthreads();
    }
    const uint64_t gi = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / (G * S);
    const int lane = (int)(threadIdx.x & 63u);
    const int sl = lane % S;                // sphere lane inside the attempt group
    const int ga = (lane / S) % G;          // attempt group
    const int gbase = lane - sl;            // first lane of this attempt group
    if (gi >= (uint64_t)n) return;          // (whole targets: blockDim is a multiple of G * S)
    const uint32_t off = (uint32_t)gi * (uint32_t)sizeof(T);
    const KAabb<T>* aabb = reinterpret_cast<const KAabb<T>*>(boxes + ca.n_boxes);
    const bool base = P.base_col >= 0;
    const T* __restrict__ qin = a.q0 ? a.q0 : q;

    T Rt[9], pt[3], trpy[3] = {T(0), T(0), T(0)};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int c = 0; c < 3; ++c) Rt[3 * r + c] = ld_soa(tgt, r + 3 * c, ldt, off);
        pt[r] = ld_soa(tgt, 9 + r, ldt, off);
    }
    if (ROWS == 6 && a.rpy_obj) {
        T kk[6];
        rpy_and_rate<KINHIP_IK_FAST_ATAN != 0>(Rt, trpy, kk);
    }
    // the scene state of this target (boxes attached to a scene mechanism): fixed during the solve
    constexpr int MG = MAXG > 0 ? MAXG : 1;
    SceneCtx<T, MG> sc;
    if constexpr (MAXG > 0) scene_frames(sc, sa, off);
    // the base of an attempt: q0's; with q_alt every restart's (k >= 1) from q_alt
    T b0[3] = {T(0), T(0), T(0)}, b1[3] = {T(0), T(0), T(0)};
    if (base)
        for (int k = 0; k < 3; ++k) {
            b0[k] = ld_soa(qin, P.base_col + k, ldq, off);
            b1[k] = a.q_alt ? ld_soa(a.q_alt, P.base_col + k, ldq, off) : b0[k];
        }
    const int L = a.attempt_len;
    int att = ga, it = ga > 0 ? ga * L + 1 : 0;  // attempt 0 from q0 at iteration 0, k >= 1 re-drawn at kL + 1
    T qs[MAXV], b[3] = {att > 0 ? b1[0] : b0[0], att > 0 ? b1[1] : b0[1], att > 0 ? b1[2] : b0[2]};
    ikt_start<T, MAXV>(P, a, qin, ldq, off, a.ibase + (int64_t)gi, att, qs);
    uint32_t held = 0;  // bit v: variable v held out of the step
    bool conv = false;
    bool done = att >= a.n_attempts;  // (groups beyond the schedule's attempts)
    int res_att = INT_MAX;            // this group's converged attempt
    // best attempt end so far (merit, attempt, state) for the no-convergence output
    T best_m = T(INFINITY), bq[MAXV], bb[3] = {T(0), T(0), T(0)}, bep = T(0), ber = T(0), bdm = T(0);
    int best_att = INT_MAX;
#pragma unroll
    for (int v = 0; v < MAXV; ++v) bq[v] = qs[v];
    T ep = T(0), er = T(0), dmin = T(INFINITY);
    const T w2 = cz.weight * cz.weight;
    const T act = cz.margin + cz.band;
#if KINHIP_IKT_SECT
    uint64_t sect_acc = 0, sect_prev = 0, sect_t0 = 0;
#endif
    const uint32_t active = P.free_mask;
    // KINHIP_IKT_LDSNE: this group's LDS region and this lane's entries of the system (row eR, column eC;
    // eC = MAXV: the right-hand side; entries past NE are read but never stored)
    // (trees of at most 12 variables: a two-arm tree's dense system of 170 entries measured 0.68 -> 0.91 ms
    // on PR2, whose replicated form folds the arms' structural zeros away)
    constexpr bool LNE = S > 1 && MAXV <= 12 && !(KINHIP_IKT_OWN) && KINHIP_IKT_LDSNE;
    using NL = IktNe<MAXV, ROWS, (NR > 0 ? NR : 1) * S>;
    constexpr int NJ = LNE ? (NL::NE + S - 1) / S : 1;
    T* ne_reg = nullptr;
    int eR[NJ], eC[NJ];
    if constexpr (LNE) {
        ne_reg = ikt_ne_lds<T, (64 / S) * NL::SIZE>() + (lane / S) * NL::SIZE;  // one region per S-lane group of the wave
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int e = sl + S * j;
            int R = 0, C = 0;
#pragma unroll
            for (int r = 0; r < MAXV; ++r)
                if (e >= NL::st(r)) {
                    R = r;
                    C = e - NL::st(r);
                }
            C = C == R + 1 ? MAXV : C;
            eR[j] = e < NL::NE ? R : 0;
            eC[j] = e < NL::NE ? C : 0;
        }
    }
    auto sdf_at = [&](T px, T py, T pz, T& d, T (&g)[3]) {  // the union (static or attached) at one point
        T xs[1] = {px}, ys[1] = {py}, zs[1] = {pz}, ds[1], gs[1][3];
        if constexpr (MAXG > 0) scene_union<T, true, 1, MG>(sc, boxes, aabb, xs, ys, zs, ds, gs, smem, use_lds);
        else union_sdf<T, true, 1>(boxes, aabb, ca.n_aabb, ca.n_boxes, xs, ys, zs, ds, gs, smem, use_lds);
        d = ds[0];
        g[0] = gs[0][0]; g[1] = gs[0][1]; g[2] = gs[0][2];
    };
    for (;;) {
        if constexpr (G > 1 || S > 1) {  // every lane of the wave is here: the loop exits wave-wide
            if constexpr (G > 1) {
                const int gm = attempt_min<G, S>(res_att);  // lowest converged attempt of the target so far
                if (!done && gm < att) done = true;
            }
            if (__ballot(!done) == 0) break;
        } else {
            if (done) break;
        }
        if (done) continue;
        KIN_IKT_STAMP(7);
        // ---- tree walk: frames, joint records, spheres ----------------------------------------------
        Fr<T> root;
        if (base) base_frame(root, b[0], b[1], b[2]);
        else set_identity(root);
        Fr<T> cur = root, Lf = root, slot[kIkcMaxSlots];
        T rz[MAXV][3], rm[MAXV][3];
#pragma unroll
        for (int v = 0; v < MAXV; ++v)
#pragma unroll
            for (int k = 0; k < 3; ++k) rz[v][k] = rm[v][k] = T(0);
        T A[MAXV][MAXV], bv[MAXV];  // lower triangle of the normal equations, right-hand side
#pragma unroll
        for (int r = 0; r < MAXV; ++r) {
            bv[r] = T(0);
#pragma unroll
            for (int c = 0; c < MAXV; ++c) A[r][c] = T(0);
        }
        // S > 1: the rows of the normal equations are accumulated by their owners -- lane sl of an attempt group
        // owns rows v = sl, sl + S, ... (Ao[o] = row o S + sl, bo[o] its right-hand side) -- and gathered into A /
        // bv for the (replicated) factorisation.  Each entry gets the same FMAs in the same order as the one-lane
        // kernel (spheres in order, then the pose rows), so the results are bit-identical for every S; a group's
        // lanes no longer each form every entry (the sphere rows and the pose rows were ~2/3 of the FMAs of an
        // iteration, on the one-wave critical path of the batch's slowest target).
        constexpr bool OWN = S > 1 && KINHIP_IKT_OWN;
        constexpr int NRO = OWN ? (MAXV + S - 1) / S : 1;
        T Ao[NRO][MAXV], bo[NRO];
#pragma unroll
        for (int o = 0; o < NRO; ++o) {
            bo[o] = T(0);
#pragma unroll
            for (int c = 0; c < MAXV; ++c) Ao[o][c] = T(0);
        }
        dmin = T(INFINITY);
        // S > 1: this lane's sphere of each round (centre, radius, the variables moving it)
        T pc[NR > 0 ? NR : 1][3], prad[NR > 0 ? NR : 1];
        uint32_t panc[NR > 0 ? NR : 1];
        if constexpr (S > 1) {
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                pc[r][0] = pc[r][1] = pc[r][2] = T(0);
                prad[r] = T(0);
                panc[r] = 0u;
            }
        }
        auto spheres = [&](const Fr<T>& f, int k0, int k1) {
            KIN_IKT_UNROLL
            for (int k = k0; k < k1; ++k) {
                const KSphere<T>& sp = sph[k];
                const uint32_t anc = sp.anc;
                const T px = fmz(f.r[0], sp.c[0], fmz(f.r[1], sp.c[1], fmz(f.r[2], sp.c[2], f.t[0])));
                const T py = fmz(f.r[3], sp.c[0], fmz(f.r[4], sp.c[1], fmz(f.r[5], sp.c[2], f.t[1])));
                const T pz = fmz(f.r[6], sp.c[0], fmz(f.r[7], sp.c[1], fmz(f.r[8], sp.c[2], f.t[2])));
                if constexpr (S == 1) {  // evaluated in the walk, rows into the system at once
                    T dr, g[3];
                    sdf_at(px, py, pz, dr, g);
                    const T d = dr - sp.r;
                    dmin = fmin(dmin, d);
                    const T viol = act - d;
                    if (viol > T(0)) {  // divergent: this lane's sphere is inside the band
                        T av[MAXV];
                        sphere_row<T, MAXV>(P, anc, px, py, pz, g, rz, rm, b, av);
                        accum_row<T, MAXV>(A, bv, av, viol, w2, anc);
                    }
                } else {  // kept by the lane that owns the sphere (k % S), evaluated after the walk
                    const int r = k / S;
                    if (k % S == sl) {
#pragma unroll
                        for (int rr = 0; rr < NR; ++rr)
                            if (rr == r) {
                                pc[rr][0] = px; pc[rr][1] = py; pc[rr][2] = pz;
                                prad[rr] = sp.r;
                                panc[rr] = anc;
                            }
                    }
                }
            }
        };
        spheres(root, P.sph_root0, P.sph_root1);
        KIN_IKT_UNROLL
        for (int s = 0; s < P.nS; ++s) {
            const KIkcStep<T>& st = St[s];
            if (st.parent == kIkcRoot) cur = root;
            else if (st.parent >= 0) pick_frame(cur, slot, st.parent);
            mul_rigid(cur, st.F);
            // _get_joint_axis (src/algorithm.jl:42-54): pre-motion world axis z and m = z x o
            const T sc0 = st.scale;
            const T zx = cur.r[2] * sc0, zy = cur.r[5] * sc0, zz = cur.r[8] * sc0;
            const T ox = cur.t[0], oy = cur.t[1], oz = cur.t[2];
#pragma unroll
            for (int v = 0; v < MAXV; ++v)
                if (v == st.var) {
                    rz[v][0] = zx; rz[v][1] = zy; rz[v][2] = zz;
                    rm[v][0] = fma(zy, oz, -(zz * oy));
                    rm[v][1] = fma(zz, ox, -(zx * oz));
                    rm[v][2] = fma(zx, oy, -(zy * ox));
                }
            motion<T, true>(cur, st.kind, st.flags, sc0, pick(qs, st.var));  // fast trig (fp32)
            if (st.save >= 0) put_frame(slot, st.save, cur);
            spheres(cur, st.sph0, st.sph1);
            if (s == P.tgt_step) Lf = cur;
        }
        link_frame(Lf, Lf, P.has_xt != 0, P.Xt);
        KIN_IKT_STAMP(1);
        uint64_t inband[NR > 0 ? NR : 1];  // S > 1: the lanes whose sphere of round r is inside the band
        if constexpr (S > 1) {
            // this lane's spheres: distance, gradient, row; then every in-band row into the system in
            // sphere order, broadcast from its lane (LNE: the rows to LDS, the system after the pose rows)
            T av[NR][MAXV], viol[NR];
            T dl = T(INFINITY);
            // every round's sphere of this lane in one pass over the union (its boxes loaded once; each
            // point's arithmetic is the one-point pass's)
            T xs[NR], ys[NR], zs[NR], ds[NR], gs[NR][3];
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                xs[r] = pc[r][0];
                ys[r] = pc[r][1];
                zs[r] = pc[r][2];
            }
            if constexpr (MAXG > 0) scene_union<T, true, NR, MG>(sc, boxes, aabb, xs, ys, zs, ds, gs, smem, use_lds);
            else union_sdf<T, true, NR>(boxes, aabb, ca.n_aabb, ca.n_boxes, xs, ys, zs, ds, gs, smem, use_lds);
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const bool valid = r * S + sl < P.n_sph;
                const T dr = ds[r];
                const T g[3] = {gs[r][0], gs[r][1], gs[r][2]};
                const T d = dr - prad[r];
                dl = valid ? fmin(dl, d) : dl;
                viol[r] = act - d;
                const bool inb = valid && viol[r] > T(0);
                sphere_row<T, MAXV>(P, panc[r], pc[r][0], pc[r][1], pc[r][2], g, rz, rm, b, av[r]);
                inband[r] = __ballot(inb);
            }
            dmin = row_group_min<S>(dl);
            KIN_IKT_STAMP(2);
            if constexpr (LNE) {  // this lane's sphere rows, zero outside the band (they then add exact zeros)
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    T* row = ne_reg + (r * S + sl) * NL::RW;
                    const bool inb = (inband[r] >> lane) & 1ull;
#pragma unroll
                    for (int v = 0; v < MAXV; ++v) {
                        row[v] = inb ? w2 * av[r][v] : T(0);
                        row[MAXV + v] = inb ? av[r][v] : T(0);
                    }
                    row[2 * MAXV] = inb ? viol[r] : T(0);
                }
            }
            KIN_IKT_UNROLL
            for (int k = 0; k < (LNE ? 0 : P.n_sph); ++k) {
                const int r = k / S, src = gbase + k % S;
                const uint32_t anc = sph[k].anc;  // (constant in the specialised kernel)
                uint64_t bal = 0;
#pragma unroll
                for (int rr = 0; rr < NR; ++rr)
                    if (rr == r) bal = inband[rr];
                if ((bal >> src) & 1ull) {  // (uniform inside the attempt group)
                    T vk = T(0), ak[MAXV];
                    // S = 16: the attempt group is one DPP row, and lane k % 16 of it broadcasts by DPP
                    auto bc = [&](T x) { return S == 16 ? row_bcast16(x, k % 16) : lane_bcast(x, src); };
#pragma unroll
                    for (int rr = 0; rr < NR; ++rr)
                        if (rr == r) {
                            vk = bc(viol[rr]);
#pragma unroll
                            for (int v = 0; v < MAXV; ++v) ak[v] = ((anc >> v) & 1u) ? bc(av[rr][v]) : T(0);
                        }
                    if constexpr (!OWN) {
                        accum_row<T, MAXV>(A, bv, ak, vk, w2, anc);
                        continue;
                    }
                    // this lane's rows (accum_row's operations on them)
                    auto own = [&](auto oc) {
                        constexpr int o = decltype(oc)::value;
                        const int v = o * S + sl;
                        if (v < MAXV && ((anc >> v) & 1u)) {  // (per lane)
                            const T wr = w2 * pick_round<o * S, S>(ak, sl);
                            bo[o] = fma(wr, vk, bo[o]);
#pragma unroll
                            for (int c = 0; c < MAXV; ++c)
                                if ((anc >> c) & 1u) Ao[o][c] = fma(wr, ak[c], Ao[o][c]);
                        }
                    };
                    own(IntC<0>());
                    if constexpr (NRO > 1) own(IntC<1>());
                    static_assert(NRO <= 2, "rows per lane (MAXV <= 2 S)");
                }
            }
        }
        KIN_IKT_STAMP(3);
        // ---- pose error, convergence, attempt ends ---------------------------------------------------
        T e[6];
        e[0] = pt[0] - Lf.t[0]; e[1] = pt[1] - Lf.t[1]; e[2] = pt[2] - Lf.t[2];
        ep = sqrt_fast(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
        er = T(0);
        T kr[6];
        if constexpr (ROWS == 6) {
            T w[3];
            if (a.rpy_obj) {
                T r[3];
                rpy_and_rate<KINHIP_IK_FAST_ATAN != 0>(Lf.r, r, kr);
#pragma unroll
                for (int k = 0; k < 3; ++k) w[k] = wrap_pi(trpy[k] - r[k]);
            } else {
                rot_error(Rt, Lf.r, w);
            }
            e[3] = w[0]; e[4] = w[1]; e[5] = w[2];
            er = sqrt_fast(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        }
        if (ep < a.tol_pos && er < a.tol_rot && dmin >= cz.margin - cz.feas) {
            conv = true;
            res_att = att;
            done = true;
            continue;
        }
        const bool last = it >= a.max_iters;  // (only the last attempt gets here)
        const bool over = !last && L > 0 && it > 0 && it % L == 0;
        if (last || over) {  // an attempt ends here: keep it if it is the best end state so far
            const T vm = fmax(cz.margin - dmin, T(0));
            T m = fma(w2 * vm, vm, fma(ep, ep, er * er));
            m = m == m ? m : T(INFINITY);  // (NaN: worst)
            if (m < best_m || best_att == INT_MAX) {
                best_m = m;
                best_att = att;
#pragma unroll
                for (int v = 0; v < MAXV; ++v) bq[v] = qs[v];
                bb[0] = b[0]; bb[1] = b[1]; bb[2] = b[2];
                bep = ep; ber = er; bdm = dmin;
            }
            if (last) {
                done = true;
                continue;
            }
            att += G;  // this group's next attempt, re-drawn
            if (att >= a.n_attempts) {
                done = true;
                continue;
            }
            it = att * L + 1;
            ikt_start<T, MAXV>(P, a, qin, ldq, off, a.ibase + (int64_t)gi, att, qs);
            for (int k = 0; k < 3; ++k) b[k] = b1[k];  // (att >= 1 here)
            held = 0;
            continue;
        }
        KIN_IKT_STAMP(4);
        // ---- pose rows: J^T J and J^T e ---------------------------------------------------------------
        // row r of J over the variables: revolute [z x p - m; z], prismatic [z; 0], base [1 0 -y'; 0 1 x'; ..]
        // (p' = p - base); with the reference objective the angular rows are d(rpy)/dq.  Accumulated row by
        // row (12 values live), each entry's FMAs in row order.
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            T Jr[MAXV];
#pragma unroll
            for (int v = 0; v < MAXV; ++v) {
                Jr[v] = T(0);
                if (!((P.tgt_mask >> v) & 1u)) continue;
                if (base && v >= P.base_col) {
                    const int k = v - P.base_col;
                    if (k == 0) Jr[v] = r == 0 ? T(1) : T(0);
                    else if (k == 1) Jr[v] = r == 1 ? T(1) : T(0);
                    else Jr[v] = r == 0 ? -(Lf.t[1] - b[1]) : r == 1 ? Lf.t[0] - b[0] : r == 5 ? T(1) : T(0);
                    continue;
                }
                const T x = rz[v][0], y = rz[v][1], z = rz[v][2];
                if ((P.prism_mask >> v) & 1u) {
                    Jr[v] = r == 0 ? x : r == 1 ? y : r == 2 ? z : T(0);
                    continue;
                }
                if (r == 0) Jr[v] = fma(y, Lf.t[2], -fma(z, Lf.t[1], rm[v][0]));
                else if (r == 1) Jr[v] = fma(z, Lf.t[0], -fma(x, Lf.t[2], rm[v][1]));
                else if (r == 2) Jr[v] = fma(x, Lf.t[1], -fma(y, Lf.t[0], rm[v][2]));
                else if (a.rpy_obj) Jr[v] = r == 3 ? fma(kr[0], x, kr[1] * y) : r == 4 ? fma(kr[2], x, kr[3] * y)
                                                                            : fma(kr[4], x, fma(kr[5], y, z));
                else Jr[v] = r == 3 ? x : r == 4 ? y : z;
            }
            if constexpr (OWN) {  // the owned rows
                auto own = [&](auto oc) {
                    constexpr int o = decltype(oc)::value;
                    const int v = o * S + sl;
                    if (v < MAXV && ((P.tgt_mask >> v) & 1u)) {  // (per lane)
                        const T jv = pick_round<o * S, S>(Jr, sl);
                        bo[o] = fma(jv, e[r], bo[o]);
#pragma unroll
                        for (int c = 0; c < MAXV; ++c)
                            if ((P.tgt_mask >> c) & 1u) Ao[o][c] = fma(jv, Jr[c], Ao[o][c]);
                    }
                };
                own(IntC<0>());
                if constexpr (NRO > 1) own(IntC<1>());
            } else if constexpr (LNE) {  // row r of J and e_r (every lane of the group the same values)
                T* jr = ne_reg + NL::JB + r * NL::JW;
#pragma unroll
                for (int v = 0; v < MAXV; ++v) jr[v] = Jr[v];
                jr[MAXV] = e[r];
            } else {
#pragma unroll
                for (int v = 0; v < MAXV; ++v)
                    if ((P.tgt_mask >> v) & 1u) bv[v] = fma(Jr[v], e[r], bv[v]);
                lower_rank1<T, MAXV>(A, Jr, Jr, P.tgt_mask);
            }
        }
        if constexpr (LNE) {
            // this lane's entries: the in-band sphere rows in sphere order, then the pose rows; then the system
            // back from every lane's entries (the group's lanes run in step: LDS accesses of a wave are in order)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            T acc[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[j] = T(0);
            // (no branch per sphere: its reads then pipeline instead of one LDS round trip per in-band sphere)
            KIN_IKT_UNROLL
            for (int k = 0; k < P.n_sph; ++k) {
                const T* row = ne_reg + k * NL::RW;
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[j] = fma(row[eR[j]], row[MAXV + eC[j]], acc[j]);
            }
#pragma unroll
            for (int i = 0; i < ROWS; ++i) {
                const T* jr = ne_reg + NL::JB + i * NL::JW;
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[j] = fma(jr[eR[j]], jr[eC[j]], acc[j]);
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                if (sl + S * j < NL::NE) ne_reg[NL::NB + sl + S * j] = acc[j];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int v = 0; v < MAXV; ++v) {
                const T* ar = ne_reg + NL::NB + NL::st(v);
#pragma unroll
                for (int c = 0; c <= v; ++c) A[v][c] = ar[c];
                bv[v] = ar[v + 1];
            }
        }
        if constexpr (OWN) {  // gather the owned rows into every lane of the group (structural zeros stay 0)
#pragma unroll
            for (int v = 0; v < MAXV; ++v) {
                const int o = v / S, ow = v % S;
                auto bc = [&](T x) { return S == 16 ? row_bcast16(x, ow) : lane_bcast(x, gbase + ow); };
                const uint32_t nz = P.nzrow[v];
                bv[v] = ((nz >> v) & 1u) ? bc(bo[o]) : T(0);
#pragma unroll
                for (int c = 0; c <= v; ++c) A[v][c] = ((nz >> c) & 1u) ? bc(Ao[o][c]) : T(0);
            }
        }
        KIN_IKT_STAMP(5);
        // ---- the step --------------------------------------------------------------------------------
        // the variables held out of the step leave the system (rows and columns 0, diagonal 1).  While no lane of
        // the wave holds one (the common case) the free set is the plan's `active` mask, a constant of the
        // specialised kernels, and the masking folds away; the same operations either way
        T y[MAXV];
        auto restrict_to = [&](uint32_t freev) {
#pragma unroll
            for (int v = 0; v < MAXV; ++v) {
                const bool fv = (freev >> v) & 1u;
#pragma unroll
                for (int c = 0; c < v; ++c)
                    if (!fv || !((freev >> c) & 1u)) A[v][c] = T(0);
                A[v][v] = fv ? A[v][v] + a.lam2 : T(1);
            }
#pragma unroll
            for (int v = 0; v < MAXV; ++v) y[v] = ((freev >> v) & 1u) ? bv[v] : T(0);
        };
        if (__builtin_constant_p(active) && __ballot(held != 0u) == 0) restrict_to(active);
        else restrict_to(active & ~held);  // (the generic kernels: one copy of the run-time masking)
        // Cholesky (in place, lower) and the two triangular solves.  fp32: the reciprocal square root of
        // each pivot (v_rsq_f32) multiplies instead of the IEEE square root and divisions (~10 instructions
        // each, on the one-wave critical path); fp64: the IEEE square root and one IEEE reciprocal per pivot,
        // which multiplies (the oracle's chol_solve; iterates to 1e-7)
        constexpr bool fast = sizeof(T) == 4;
        T ip[MAXV];
#pragma unroll
        for (int j = 0; j < MAXV; ++j) {
            T d = A[j][j];
#pragma unroll
            for (int k = 0; k < j; ++k) d = fnz(A[j][k], A[j][k], d);
            T id;
            if constexpr (fast) {
                id = rsqrt_fast(d);
                ip[j] = id;
            } else {
                d = sqrt_t(d);
                A[j][j] = d;
                id = T(1) / d;
                ip[j] = id;
            }
#pragma unroll
            for (int r = j + 1; r < MAXV; ++r) {
                T sm = A[r][j];
#pragma unroll
                for (int k = 0; k < j; ++k) sm = fnz(A[r][k], A[j][k], sm);
                A[r][j] = mul0(sm, id);
            }
        }
#pragma unroll
        for (int r = 0; r < MAXV; ++r) {
            T sm = y[r];
#pragma unroll
            for (int k = 0; k < r; ++k) sm = fnz(A[r][k], y[k], sm);
            y[r] = sm * ip[r];
        }
#pragma unroll
        for (int r = MAXV - 1; r >= 0; --r) {
            T sm = y[r];
#pragma unroll
            for (int k = r + 1; k < MAXV; ++k) sm = fnz(A[k][r], y[k], sm);
            y[r] = sm * ip[r];
        }
        KIN_IKT_STAMP(6);
        T mx = T(0);
        uint32_t nh = 0;
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            if (!((active >> v) & 1u)) continue;
            if ((P.joint_mask >> v) & 1u) {
                const bool was = (held >> v) & 1u;
                const T dir = was ? bv[v] : y[v];  // held: the descent direction J^T e + ...
                // (bitwise, not short-circuit: selects instead of ~20 exec-mask instructions per joint)
                const bool out = ((qs[v] <= P.vlo[v]) & (dir < T(0))) | ((qs[v] >= P.vhi[v]) & (dir > T(0)));
                nh |= (uint32_t)out << v;
                y[v] = was ? T(0) : y[v];
            }
            mx = fmax(mx, fabs(y[v]));
        }
        held = nh;
        const T sc = mx > a.max_step ? a.max_step / mx : T(1);
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            if (!((active >> v) & 1u)) continue;
            if ((P.joint_mask >> v) & 1u) qs[v] = fmin(fmax(fma(sc, y[v], qs[v]), P.vlo[v]), P.vhi[v]);
            else if (base && v >= P.base_col) {
                const int k = v - P.base_col;
                const T nb = fma(sc, y[v], b[k]);
                b[0] = k == 0 ? nb : b[0];
                b[1] = k == 1 ? nb : b[1];
                b[2] = k == 2 ? nb : b[2];
            }
        }
        ++it;
    }
    // ---- outputs: the lowest converged attempt, else the best attempt end ----------------------------
    bool write = true;
    if constexpr (G > 1) {
        const int gm = attempt_min<G, S>(res_att);
        if (gm != INT_MAX) {
            write = res_att == gm;
        } else {
            const T mm = attempt_min_t<G, S>(best_m);
            const int am = attempt_min<G, S>(best_m == mm ? best_att : INT_MAX);
            write = best_att == am;
        }
    }
    if (!write || sl != 0) return;
    if (!conv) {
#pragma unroll
        for (int v = 0; v < MAXV; ++v) qs[v] = bq[v];
        b[0] = bb[0]; b[1] = bb[1]; b[2] = bb[2];
        ep = bep; er = ber; dmin = bdm;
    }
    for (int v = 0; v < P.n_q; ++v) st_soa(q, v, ldq, off, pick(qs, v));
    if (base)
        for (int k = 0; k < 3; ++k) st_soa(q, P.base_col + k, ldq, off, b[k]);
    if (iters) iters[gi] = conv ? it : a.max_iters + 1;
#if KINHIP_IKT_SECT
    {
        uint64_t t_;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
        ep = (T)(double)sect_acc;
        er = (T)(double)(t_ - sect_t0);
    }
#endif
    if (err) {
        st_soa(err, 0, lde, off, ep);
        st_soa(err, 1, lde, off, er);
        st_soa(err, 2, lde, off, dmin);
    }
}

}  // namespace
}  // namespace kinhip

#pragma clang fp contract(fast)  // (the translation unit's default again: -ffp-contract=fast-honor-pragmas)
