// kinhip_ikc_dev.h -- device body of k_ik_coll: batched collision-aware IK, the second stage of
// inverse_kinematics!(m, link, joints, target, sscc, sdf; use_bistage) (src/inverse_kinematics.jl:
// 1-21): the pose objective subject to IneqConst(sscc, joints, sdf, 1, margin) (src/planning.jl:55-68,
// every swept sphere at least `margin` from the UnionSDF).  Included by kinhip_ik.hip (generic kernel)
// and embedded in the run-time specialised source (kinhip_jit.cpp).  gfx950 only.
#pragma once
#include "kinhip_coll_dev.h"
#include "kinhip_ik_dev.h"

namespace kinhip {
namespace {

// Constraint handling of k_ik_coll (kin_ik_coll_params)
template <typename T>
struct IkcArgsT {
    T margin;  // IneqConst margin (the reference's stage 2 uses 0.02)
    T band;    // a sphere with d < margin + band is pushed towards margin + band
    T weight;  // weight of a sphere's row against the pose rows
    T feas;    // converged only when every sphere has d >= margin - feas
};

// G lanes per target (aligned lane groups, G = 1 or 4): lane `slot` of a group runs attempts slot,
// slot + G, ... of the restart schedule of k_ik_dls side by side with the others, stops once a lower
// attempt of its target has converged (group_min by DPP every iteration), and the lowest converged
// attempt (else the last one) writes.  Every lane's arithmetic is the sequential schedule's (G = 1:
// attempts in sequence on one lane), so the results are identical for G = 1 and 4; a small batch (the
// bistage solve's few thousand targets are a fraction of a wave per SIMD) gains the parallelism and
// a wave no longer lasts as long as the sum of its slowest target's attempts.  Per iteration:
// FK with the joint records, every sphere's centre and UnionSDF distance + analytic gradient on the
// way (k_coll's union_sdf), then ONE damped Gauss-Newton step on the normal equations over the chain's
// joints (+ base):
//     (J^T J + sum_k w^2 a_k^T a_k + lambda^2 I) dq = J^T e + sum_k w^2 a_k^T (margin + band - d_k)
// where the sum runs over the spheres with d_k < margin + band and a_k = grad sdf^T J_k (1 x n, the
// IneqConst row of sphere k).  A sphere row is a one-sided penalty: it pushes only while the sphere is
// inside the band, so in the null space of the pose task the arm moves out to the band and the pose
// error is driven to zero; the attempt has converged when |dp| < tol_pos, |rot| < tol_rot and every
// sphere has d >= margin - feas.  Joint limits: a joint that sits on a limit and is pushed further out
// (by this step if it was free, by the gradient J^T e + ... if it was held) is held out of the next
// step (row / column of the system replaced by the identity); q is clamped to the limits.
template <typename T, int MAXA, int ROWS, int G>
__device__ __forceinline__ void ikc_body(const KProg<T>& P, const KStep<T>* __restrict__ S,
                                         const KSphere<T>* __restrict__ sph, const KBox<T>* __restrict__ boxes,
                                         const CollArgs& ca, const IkcArgsT<T>& cz, const IkArgsT<T>& a,
                                         const T* __restrict__ tgt, int64_t ldt, T* __restrict__ q, int64_t ldq,
                                         int64_t n, int32_t* __restrict__ iters, T* __restrict__ err, int64_t lde,
                                         unsigned char* smem) {
    const bool use_lds = ca.n_boxes <= kCollLdsBoxes;  // argmin box gathers from LDS (k_coll)
    if (use_lds) {
        const int words = ca.n_boxes * (int)(sizeof(KBox<T>) / 16);
        for (int w = (int)threadIdx.x; w < words; w += (int)blockDim.x)
            reinterpret_cast<uint4*>(smem)[w] = reinterpret_cast<const uint4*>(boxes)[w];
        __syncthreads();
    }
    static_assert(G == 1 || G == 2 || G == 4 || G == 8, "lane groups inside a DPP row");
    const uint64_t gi = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    const int slot = (int)(threadIdx.x % G);
    if (gi >= (uint64_t)n) return;  // (whole lane groups: blockDim is a multiple of G)
    const uint32_t off = (uint32_t)gi * (uint32_t)sizeof(T);
    const KAabb<T>* aabb = reinterpret_cast<const KAabb<T>*>(boxes + ca.n_boxes);
    const bool base = (P.flags & PF_BASE) != 0;
    constexpr int ND = MAXA + 3;  // chain steps, then the base (x, y, theta)
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
        rpy_and_rate(Rt, trpy, kk);
    }
    T b0[3] = {T(0), T(0), T(0)};
    if (base)
        for (int k = 0; k < 3; ++k) b0[k] = ld_soa(qin, P.base_col + k, ldq, off);
    T qs[MAXA], b[3] = {b0[0], b0[1], b0[2]};
    const int L = a.attempt_len;
    // this lane's first attempt: attempt 0 from q0 at iteration 0, attempt k >= 1 re-drawn at kL + 1
    int att = slot, it = slot > 0 ? slot * L + 1 : 0;
    ik_start_attempt<T, MAXA>(S, a, qin, ldq, off, a.ibase + (int64_t)gi, att, qs);
    uint32_t held = 0;  // bit v: variable v (step v, base MAXA + k) held out of the step
    bool conv = false, final_lane = false;
    bool done = att >= a.n_attempts;  // (lanes beyond the schedule's attempts)
    int res_att = INT_MAX;            // this lane's converged attempt
    T ep = T(0), er = T(0), dmin = T(INFINITY);
    const T w2 = cz.weight * cz.weight;
    const T act = cz.margin + cz.band;
    for (;;) {
        if constexpr (G > 1) {  // every lane of the wave is here: the loop exits wave-wide
            const int gm = group_min<G>(res_att);  // lowest converged attempt of the target so far
            if (!done && gm < att) done = true;
            if (__ballot(!done) == 0) break;
        } else {
            if (done) break;
        }
        if (done) continue;
        // ---- FK, records, spheres -------------------------------------------------------------
        Fr<T> f;
        if (base) base_frame(f, b[0], b[1], b[2]);
        else set_identity(f);
        T ro[MAXA][3], rz[MAXA][3];
        T A[ND][ND], bv[ND];  // lower triangle of the normal equations, right-hand side
#pragma unroll
        for (int r = 0; r < ND; ++r) {
            bv[r] = T(0);
#pragma unroll
            for (int c = 0; c < ND; ++c) A[r][c] = T(0);
        }
        dmin = T(INFINITY);
        // sphere rows: a_v = g . (z_v x (c - o_v)) = z_v . (c x g) - g . m_v with m_v = z_v x o_v (k_coll)
        auto sphere_rows = [&](int s_last, int k0, int k1) {
            for (int k = k0; k < k1; ++k) {
                const KSphere<T>& sp = sph[k];
                T px[1], py[1], pz[1], ds[1], g[1][3];
                px[0] = fmz(f.r[0], sp.c[0], fmz(f.r[1], sp.c[1], fmz(f.r[2], sp.c[2], f.t[0])));
                py[0] = fmz(f.r[3], sp.c[0], fmz(f.r[4], sp.c[1], fmz(f.r[5], sp.c[2], f.t[1])));
                pz[0] = fmz(f.r[6], sp.c[0], fmz(f.r[7], sp.c[1], fmz(f.r[8], sp.c[2], f.t[2])));
                union_sdf<T, true, 1>(boxes, aabb, ca.n_aabb, ca.n_boxes, px, py, pz, ds, g, smem, use_lds);
                const T d = ds[0] - sp.r;
                dmin = fmin(dmin, d);
                const T viol = act - d;
                if (viol > T(0)) {  // divergent: this lane's sphere is inside the band
                    const T w0 = fma(py[0], g[0][2], -(pz[0] * g[0][1]));
                    const T w1 = fma(pz[0], g[0][0], -(px[0] * g[0][2]));
                    const T w3 = fma(px[0], g[0][1], -(py[0] * g[0][0]));
                    T av[ND];
#pragma unroll
                    for (int v = 0; v < ND; ++v) av[v] = T(0);
#pragma unroll
                    for (int j = 0; j < MAXA; ++j) {
                        if (j <= s_last && (S[j].flags & SF_REC) && S[j].qcol >= 0) {
                            if (S[j].jkind == MOT_PRISM)
                                av[j] = fma(g[0][0], rz[j][0], fma(g[0][1], rz[j][1], g[0][2] * rz[j][2]));
                            else
                                av[j] = fma(rz[j][0], w0, fma(rz[j][1], w1, fma(rz[j][2], w3,
                                        -fma(g[0][0], ro[j][0], fma(g[0][1], ro[j][1], g[0][2] * ro[j][2])))));
                        }
                    }
                    if (base) {  // base columns [1 0 -y; 0 1 x; 0 0 0] of the sphere point
                        av[MAXA] = g[0][0];
                        av[MAXA + 1] = g[0][1];
                        av[MAXA + 2] = fma(-g[0][0], py[0] - b[1], g[0][1] * (px[0] - b[0]));
                    }
#pragma unroll
                    for (int r = 0; r < ND; ++r) {
                        if (r >= MAXA && !base) continue;
                        bv[r] = fma(w2 * av[r], viol, bv[r]);
#pragma unroll
                        for (int c = 0; c <= r; ++c) A[r][c] = fma(w2 * av[r], av[c], A[r][c]);
                    }
                }
            }
        };
        sphere_rows(-1, P.sph_root0, P.sph_root1);
#pragma unroll
        for (int s = 0; s < MAXA; ++s) {
            step_a<T, true>(f, S[s], qs[s], ro[s], rz[s]);  // fast trig (fp32)
            const T o0 = ro[s][0], o1 = ro[s][1], o2 = ro[s][2];  // m_s = z_s x o_s (held in ro)
            ro[s][0] = fma(rz[s][1], o2, -(rz[s][2] * o1));
            ro[s][1] = fma(rz[s][2], o0, -(rz[s][0] * o2));
            ro[s][2] = fma(rz[s][0], o1, -(rz[s][1] * o0));
            sphere_rows(s, S[s].sph0, S[s].sph1);
        }
        Fr<T> Lf;
        link_frame(Lf, f, P.last_has_x != 0, P.Xlast);
        // ---- pose error and convergence --------------------------------------------------------
        T e[6];
        e[0] = pt[0] - Lf.t[0]; e[1] = pt[1] - Lf.t[1]; e[2] = pt[2] - Lf.t[2];
        ep = sqrt_fast(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
        er = T(0);
        T kr[6];
        if constexpr (ROWS == 6) {
            T w[3];
            if (a.rpy_obj) {
                T r[3];
                rpy_and_rate(Lf.r, r, kr);
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
        if (it >= a.max_iters) {  // (only the last attempt gets here)
            final_lane = true;
            done = true;
            continue;
        }
        if (L > 0 && it > 0 && it % L == 0) {  // attempt over: this lane's next one, re-drawn
            att += G;
            if (att >= a.n_attempts) {
                final_lane = att - G == a.n_attempts - 1;
                done = true;
                continue;
            }
            it = att * L + 1;
            ik_start_attempt<T, MAXA>(S, a, qin, ldq, off, a.ibase + (int64_t)gi, att, qs);
            b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2];
            held = 0;
            continue;
        }
        // ---- pose rows: J^T J and J^T e ---------------------------------------------------------
        // column of step s: revolute [z x (p - o); z] = [z x p - m; z] (m = z x o held in ro),
        // prismatic [z; 0]; with the reference objective the angular rows are d(rpy)/dq
        T Jc[ND][ROWS];
#pragma unroll
        for (int s = 0; s < MAXA; ++s) {
#pragma unroll
            for (int r = 0; r < ROWS; ++r) Jc[s][r] = T(0);
            if (!((S[s].flags & SF_REC) && S[s].qcol >= 0)) continue;
            const T x = rz[s][0], y = rz[s][1], z = rz[s][2];
            if (S[s].jkind == MOT_PRISM) {
                Jc[s][0] = x; Jc[s][1] = y; Jc[s][2] = z;
                continue;
            }
            Jc[s][0] = fma(y, Lf.t[2], -fma(z, Lf.t[1], ro[s][0]));
            Jc[s][1] = fma(z, Lf.t[0], -fma(x, Lf.t[2], ro[s][1]));
            Jc[s][2] = fma(x, Lf.t[1], -fma(y, Lf.t[0], ro[s][2]));
            if constexpr (ROWS == 6) {
                if (a.rpy_obj) {
                    Jc[s][3] = fma(kr[0], x, kr[1] * y);
                    Jc[s][4] = fma(kr[2], x, kr[3] * y);
                    Jc[s][5] = fma(kr[4], x, fma(kr[5], y, z));
                } else {
                    Jc[s][3] = x; Jc[s][4] = y; Jc[s][5] = z;
                }
            }
        }
        if (base) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int r = 0; r < ROWS; ++r) Jc[MAXA + k][r] = T(0);
            Jc[MAXA][0] = T(1);
            Jc[MAXA + 1][1] = T(1);
            Jc[MAXA + 2][0] = -(Lf.t[1] - b[1]);
            Jc[MAXA + 2][1] = Lf.t[0] - b[0];
            if constexpr (ROWS == 6) Jc[MAXA + 2][5] = T(1);
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int r = 0; r < ROWS; ++r) Jc[MAXA + k][r] = T(0);
        }
#pragma unroll
        for (int v = 0; v < ND; ++v) {
            T s = bv[v];
#pragma unroll
            for (int r = 0; r < ROWS; ++r) s = fma(Jc[v][r], e[r], s);
            bv[v] = s;
#pragma unroll
            for (int c = 0; c <= v; ++c) {
                T x = A[v][c];
#pragma unroll
                for (int r = 0; r < ROWS; ++r) x = fma(Jc[v][r], Jc[c][r], x);
                A[v][c] = x;
            }
        }
        // ---- the step -------------------------------------------------------------------------
        uint32_t active = 0;  // variables of the system: recorded chain steps with a column, base
#pragma unroll
        for (int s = 0; s < MAXA; ++s)
            if ((S[s].flags & SF_REC) && S[s].qcol >= 0) active |= 1u << s;
        if (base) active |= 7u << MAXA;
        const uint32_t freev = active & ~held;
#pragma unroll
        for (int v = 0; v < ND; ++v) {
            const bool fv = (freev >> v) & 1u;
#pragma unroll
            for (int c = 0; c < v; ++c)
                if (!fv || !((freev >> c) & 1u)) A[v][c] = T(0);
            A[v][v] = fv ? A[v][v] + a.lam2 : T(1);
        }
        T y[ND];
#pragma unroll
        for (int v = 0; v < ND; ++v) y[v] = ((freev >> v) & 1u) ? bv[v] : T(0);
        // Cholesky of the ND x ND system (in place, lower) and the two triangular solves
#pragma unroll
        for (int j = 0; j < ND; ++j) {
            T d = A[j][j];
#pragma unroll
            for (int k = 0; k < j; ++k) d -= A[j][k] * A[j][k];
            d = sqrt_t(d);
            A[j][j] = d;
            const T id = T(1) / d;
#pragma unroll
            for (int r = j + 1; r < ND; ++r) {
                T sm = A[r][j];
#pragma unroll
                for (int k = 0; k < j; ++k) sm -= A[r][k] * A[j][k];
                A[r][j] = sm * id;
            }
        }
#pragma unroll
        for (int r = 0; r < ND; ++r) {
            T sm = y[r];
#pragma unroll
            for (int k = 0; k < r; ++k) sm -= A[r][k] * y[k];
            y[r] = sm / A[r][r];
        }
#pragma unroll
        for (int r = ND - 1; r >= 0; --r) {
            T sm = y[r];
#pragma unroll
            for (int k = r + 1; k < ND; ++k) sm -= A[k][r] * y[k];
            y[r] = sm / A[r][r];
        }
        T mx = T(0);
        uint32_t nh = 0;
#pragma unroll
        for (int s = 0; s < MAXA; ++s) {
            if (!((active >> s) & 1u)) continue;
            const bool was = (held >> s) & 1u;
            const T dir = was ? bv[s] : y[s];  // held: the descent direction J^T e + ...
            if ((qs[s] <= S[s].lo && dir < T(0)) || (qs[s] >= S[s].hi && dir > T(0))) nh |= 1u << s;
            if (was) y[s] = T(0);
            mx = fmax(mx, fabs(y[s]));
        }
        if (base)
            for (int k = 0; k < 3; ++k) mx = fmax(mx, fabs(y[MAXA + k]));
        held = nh;
        const T sc = mx > a.max_step ? a.max_step / mx : T(1);
#pragma unroll
        for (int s = 0; s < MAXA; ++s) qs[s] = fmin(fmax(qs[s] + sc * y[s], S[s].lo), S[s].hi);
        if (base)
            for (int k = 0; k < 3; ++k) b[k] = b[k] + sc * y[MAXA + k];
        ++it;
    }
    // ---- outputs: the lowest converged attempt of the target, else the last one --------------------
    if constexpr (G > 1) {
        const int gm = group_min<G>(res_att);
        if (gm != INT_MAX ? res_att != gm : !final_lane) return;
    }
#pragma unroll
    for (int s = 0; s < MAXA; ++s) {
        const int32_t c = S[s].qcol;
        if (c >= 0) st_soa(q, c, ldq, off, qs[s]);
    }
    if (base)
        for (int k = 0; k < 3; ++k) st_soa(q, P.base_col + k, ldq, off, b[k]);
    if (iters) iters[gi] = conv ? it : a.max_iters + 1;
    if (err) {
        st_soa(err, 0, lde, off, ep);
        st_soa(err, 1, lde, off, er);
        st_soa(err, 2, lde, off, dmin);
    }
}

}  // namespace
}  // namespace kinhip
