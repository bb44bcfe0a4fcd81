// kinhip_fk_dev.h -- device body of k_fk (batched get_transform + get_jacobian!).
// Included by kinhip_fk.hip (generic kernel) and embedded in the run-time
// specialised source (kinhip_jit.cpp).  gfx950 only.
#pragma once
#include "kinhip_device.h"

namespace kinhip {
namespace {

// --------------------------------------------------------------------------
// k_fk: batched get_transform (any set of links) + get_jacobian! of one link
// --------------------------------------------------------------------------
// The body is shared by the generic kernel (program in device memory, read
// through the scalar cache) and the plan-specialised kernels compiled at run
// time (kinhip_jit.cpp: P and S are constexpr, so every step's F, X, kind and
// column mask fold into the instruction stream).
// angles (and base pose) of unit b (256 configurations) for this lane
template <typename T, int MAXA>
__device__ __forceinline__ void fk_load(const KProg<T>& P, const KStep<T>* __restrict__ S, const T* __restrict__ q,
                                        int64_t ldq, const Tiling& tl, uint32_t b, T (&qa)[MAXA], T (&bq)[3]) {
    const uint32_t t = b / tl.tile_blocks;
    const T* qt = q ? q + (int64_t)t * tl.tsq : q;
    const uint32_t off = ((b - t * tl.tile_blocks) * blockDim.x + threadIdx.x) * (uint32_t)sizeof(T);
    bq[0] = bq[1] = bq[2] = T(0);
    if (P.flags & PF_BASE)
        for (int k = 0; k < 3; ++k) bq[k] = ld_soa(qt, P.base_col + k, ldq, off);
    // every phase-A angle load issued up front (independent, coalesced)
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const int32_t c = S[s].qcol;
        qa[s] = c >= 0 ? ld_soa(qt, c, ldq, off) : T(0);
    }
}

template <typename T, int MAXA>
__device__ __forceinline__ void fk_one(const KProg<T>& P, const KStep<T>* __restrict__ S, T* slots,
                                       const T* __restrict__ q, int64_t ldq, T* __restrict__ poses, int64_t ldp,
                                       T* __restrict__ jac, int64_t ldj, const Tiling& tl, uint32_t b,
                                       const T (&qa)[MAXA], const T (&bq)[3]);

// STRIDE: grid-strided units with the next unit's angles prefetched (launch_fk picks it for batches
// far larger than the Infinity Cache; specialised kernels only)
template <typename T, int MAXA, bool STRIDE = false>
__device__ __forceinline__ void fk_body(const KProg<T>& P, const KStep<T>* __restrict__ S, T* slots,
                                        const T* __restrict__ q, int64_t ldq, int64_t n, T* __restrict__ poses,
                                        int64_t ldp, T* __restrict__ jac, int64_t ldj, const Tiling& tl) {
    const uint32_t B = blockDim.x, tid = threadIdx.x;
    T qa[MAXA], bq[3];
    if constexpr (STRIDE) {
    // grid-strided units of B configurations: a lane evaluates several, and the next unit's
    // angles are loaded before this one is computed and stored (no barrier below: lanes past n
    // only skip their own work)
    const uint32_t units = (uint32_t)((n + B - 1) / B);
    uint32_t b = blockIdx.x;
    if (b >= units) return;
    if ((uint64_t)b * B + tid < (uint64_t)n) fk_load<T, MAXA>(P, S, q, ldq, tl, b, qa, bq);
    for (;;) {
        const uint32_t bn = b + gridDim.x;
        T qn[MAXA], bqn[3];
        const bool more = bn < units;
        if (more && (uint64_t)bn * B + tid < (uint64_t)n) fk_load<T, MAXA>(P, S, q, ldq, tl, bn, qn, bqn);
        if ((uint64_t)b * B + tid < (uint64_t)n)
            fk_one<T, MAXA>(P, S, slots, q, ldq, poses, ldp, jac, ldj, tl, b, qa, bq);
        if (!more) break;
        b = bn;
#pragma unroll
        for (int s = 0; s < MAXA; ++s) qa[s] = qn[s];
        bq[0] = bqn[0]; bq[1] = bqn[1]; bq[2] = bqn[2];
    }
    } else {
    const uint32_t b = config_block();
    if ((uint64_t)b * B + tid >= (uint64_t)n) return;  // no block-wide barrier below: LDS slots are per lane
    fk_load<T, MAXA>(P, S, q, ldq, tl, b, qa, bq);
    fk_one<T, MAXA>(P, S, slots, q, ldq, poses, ldp, jac, ldj, tl, b, qa, bq);
    }
}

// one configuration per lane of unit b
template <typename T, int MAXA>
__device__ __forceinline__ void fk_one(const KProg<T>& P, const KStep<T>* __restrict__ S, T* slots,
                                       const T* __restrict__ q, int64_t ldq, T* __restrict__ poses, int64_t ldp,
                                       T* __restrict__ jac, int64_t ldj, const Tiling& tl, uint32_t b,
                                       const T (&qa)[MAXA], const T (&bq)[3]) {
    const int B = blockDim.x, tid = threadIdx.x;
#ifdef KINHIP_JIT
    // specialised kernels: every slot index is a constant, so branch frames live in registers
    // (the array is scalar-replaced) instead of per-lane LDS slots
    Fr<T> rslot[kMaxSlots];
#define KIN_SLOT_STORE(sl, fr) rslot[sl] = (fr)
#define KIN_SLOT_LOAD(sl, fr) (fr) = rslot[sl]
#else
#define KIN_SLOT_STORE(sl, fr) slot_store(slots, (sl), B, tid, (fr))
#define KIN_SLOT_LOAD(sl, fr) slot_load(slots, (sl), B, tid, (fr))
#endif
    // tiled SoA: this workgroup's tile (wave-uniform) moves the array bases; lanes keep a 32-bit offset
    const uint32_t t = b / tl.tile_blocks;
    if (q) q += (int64_t)t * tl.tsq;
    if (poses) poses += (int64_t)t * tl.tsp;
    if (jac) jac += (int64_t)t * tl.tsj;
    const uint32_t i = (b - t * tl.tile_blocks) * (uint32_t)B + tid;
    const uint32_t off = i * (uint32_t)sizeof(T);
    Sink<T> sk;
    sk.off = off;

    const bool base = (P.flags & PF_BASE) != 0;
    const T bx = bq[0], by = bq[1], bth = bq[2];
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
        if (st.save >= 0) KIN_SLOT_STORE(st.save, f);
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
#ifdef KINHIP_JIT
#pragma unroll
#endif
    for (int s = P.nA; s < P.nS; ++s) {
        const KStep<T>& st = S[s];
        const int32_t ld = st.load;
        if (ld == LOAD_ROOT) f = root;
        else if (ld >= 0) KIN_SLOT_LOAD(ld, f);
        mul_rigid(f, st.F);
        if (st.kind != MOT_NONE) motion(f, st.kind, st.flags, st.scale, ld_soa(q, st.qcol, ldq, off));
        if (st.out >= 0) {
            Fr<T> L;
            link_frame(L, f, (st.flags & SF_HAS_X) != 0, st.X);
            store_pose(sk, poses, st.out, ldp, L);
        }
        if (st.save >= 0) KIN_SLOT_STORE(st.save, f);
    }
}

#undef KIN_SLOT_STORE
#undef KIN_SLOT_LOAD
}  // namespace
}  // namespace kinhip
