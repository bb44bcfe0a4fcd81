// kinhip_fk.hip -- k_fk (batched get_transform + get_jacobian!) and k_pose_residual.
// (gfx950 only; shared helpers in kinhip_device.h)
#include "kinhip_device.h"

namespace kinhip {
namespace {

// --------------------------------------------------------------------------
// k_fk: batched get_transform (any set of links) + get_jacobian! of one link
// --------------------------------------------------------------------------
template <typename T, int MAXA>
__global__ __launch_bounds__(256) void k_fk(const KProg<T> P, const KStep<T>* __restrict__ S,
                                            const T* __restrict__ q, int64_t ldq, int64_t n,
                                            T* __restrict__ poses, int64_t ldp, T* __restrict__ jac,
                                            int64_t ldj, const Tiling tl) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* slots = reinterpret_cast<T*>(smem);
    const int B = blockDim.x, tid = threadIdx.x;
    const uint32_t b = config_block();
    if ((uint64_t)b * (uint32_t)B + tid >= (uint64_t)n) return;  // no block-wide barrier below: LDS slots are per lane
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

}  // namespace

template <typename T>
hipError_t launch_fk(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const T* q, int64_t ldq,
                     int64_t n, T* poses, int64_t ldp, T* jac, int64_t ldj, const TileArgs& ta, hipStream_t st) {
    // plain SoA (tile >= n): chunks are element offsets along the rows; tiled: whole tiles per chunk
    const bool tiled = ta.tile < n;
    const int64_t chunk = tiled ? (kChunk / ta.tile) * ta.tile : kChunk;
    Tiling tl{tiled ? (uint32_t)(ta.tile / g.block) : 0xffffffffu, ta.tsq, ta.tsp, ta.tsj};
    for (int64_t s0 = 0; s0 < n; s0 += chunk) {
        const int64_t c = std::min(chunk, n - s0);
        const dim3 grid(grid_of(c, g.block)), block(g.block);
        const int64_t tq = tiled ? (s0 / ta.tile) * ta.tsq : s0, tp = tiled ? (s0 / ta.tile) * ta.tsp : s0,
                      tj = tiled ? (s0 / ta.tile) * ta.tsj : s0;
        const T* qc = q ? q + tq : q;
        T* pc = poses ? poses + tp : poses;
        T* jc = jac ? jac + tj : jac;
#define KIN_FK_LAUNCH(MA) \
        hipLaunchKernelGGL((k_fk<T, MA>), grid, block, g.lds, st, P, steps, qc, ldq, c, pc, ldp, jc, ldj, tl)
        KIN_MAXA_DISPATCH(g.maxA, KIN_FK_LAUNCH)
#undef KIN_FK_LAUNCH
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
                                     int64_t, T*, int64_t, T*, int64_t, const TileArgs&, hipStream_t);       \
    template hipError_t launch_pose_residual<T>(const T*, int64_t, const T*, int64_t, int64_t, int, T*, int64_t, \
                                                hipStream_t);
KIN_INSTANTIATE(float)
KIN_INSTANTIATE(double)

}  // namespace kinhip
