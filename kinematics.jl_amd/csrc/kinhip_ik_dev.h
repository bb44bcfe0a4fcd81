// kinhip_ik_dev.h -- device bodies of k_ik_dls (batched DLS IK with restarts)
// and k_nakamura.  Included by kinhip_ik.hip (generic kernels) and embedded
// in the run-time specialised source (kinhip_jit.cpp).  gfx950 only.
#pragma once
#include "kinhip_device.h"

namespace kinhip {
namespace {

#ifndef KINHIP_IK_NARROW
#define KINHIP_IK_NARROW 0  // 1: narrow SoA addressing (ldn_soa) in k_ik_dls, see kinhip_device.h
#endif
#ifndef KINHIP_IK_PK
#define KINHIP_IK_PK 1  // fp32: packed FMAs for J W J^T (ik_body)
#endif
#ifndef KINHIP_IK_FAST_ATAN
#define KINHIP_IK_FAST_ATAN 1  // fp32: polynomial atan2 for the rotation error's angle (rot_error)
#endif
// fp32: the damped solve (J W J^T + lambda^2 I, its Cholesky, the two triangular solves and dq = J^T y)
// in fp64 from the fp32 Jacobian.  Forming J J^T in fp32 errs by ~eps |J|^2 = 2.4e-7 against
// lambda^2 = 1e-4, and at a singular arm (Fetch at q = 0: rank 4) y carries ~e / lambda^2 in the null
// directions that J^T y cancels: an fp32 solve moves dq by up to 2e-3 rad against the fp64 oracle's,
// the J rounding alone by 1e-6 (tools/ik_fp32_solve_error.py).  0: the fp32 solve (A/B build).  2: the
// fp32 factorisation and solve plus one step of iterative refinement whose residual
// e - (J W J^T + lambda'^2 I) y is formed in fp64 from J itself (J^T y, then J (W J^T y)), never from
// the rounded J J^T: the fp32 factor contracts the error by ~eps kappa ~ 1e-3 per step.  3: the fp64
// solve for the first KINHIP_IK_F64_ITERS iterations of attempt 0 only -- the attempt that starts from
// the caller's q0, which for config 4 (and any caller starting from a zero / home pose) is a singular
// arm (Fetch at q = 0: rank 4) -- and the fp32 solve everywhere else.  Along config-4 trajectories the
// fp32 solve's step error (fp32 normal equations vs fp64, the same fp32 J) is <= 8.4e-4 at iteration 0,
// 5.5e-4 at 1, 4.3e-4 at 2 and <= 1.8e-4 from iteration 3 on, 99.4% of the lanes <= 1e-5 there; restart
// attempts start from random angles (tools/ik_cond_explore.py).  The choice is a function of the lane's
// own attempt and iteration, so every lane layout / schedule still gives identical results, and phase 1
// of the two-phase schedule (every lane at the same iteration) takes one path per wave.
#ifndef KINHIP_IK_F64SOLVE
#define KINHIP_IK_F64SOLVE 3
#endif
#ifndef KINHIP_IK_F64_ITERS
#define KINHIP_IK_F64_ITERS 3
#endif
// ... and with KINHIP_IK_F64SOLVE = 3 the fp64 solve everywhere when lambda^2 is below this: the
// analysis above rests on lambda^2 = 1e-4 against the fp32 normal equations' ~eps |J|^2 = 2.4e-7; a smaller
// damping (down to lambda = 0, which kin_ik_params accepts) leaves the fp32 factorisation of a near-singular
// arm without that margin (NaN pivots at lambda = 0).  A uniform kernel argument: one path per wave.
#ifndef KINHIP_IK_F32SOLVE_MIN_LAM2
#define KINHIP_IK_F32SOLVE_MIN_LAM2 0.99e-4
#endif
// Contraction only inside one expression (a * b + c): the specialised kernels (hiprtc) fold constants
// into the instruction stream, and fusing across statements would then differ from the generic ones
#ifndef KINHIP_CONTRACT_FAST
#define KINHIP_CONTRACT_FAST 0  // A/B only (KINHIP_JIT_DEFS): fusion across statements, spec != generic
#endif
#if KINHIP_CONTRACT_FAST
#pragma clang fp contract(fast)
#else
#pragma clang fp contract(on)
#endif
// Diagnostic section stamps (tools only: KINHIP_JIT_DEFS=-DKINHIP_IK_SECT=<k> in the A/B build): the
// cycles of iteration section k (1 FK, 2 errors + checks, 3 Jacobian + J W J^T, 4 Cholesky + solves,
// 5 dq + active set, 6 step, 7 loop top) summed over the lane's iterations replace err row 0 and the
// lane's cycles from its first iteration to its write replace err row 1.  Never in a product build.
#ifndef KINHIP_IK_SECT
#define KINHIP_IK_SECT 0
#endif
#if KINHIP_IK_SECT
__device__ __forceinline__ uint64_t ik_stamp() {
    uint64_t t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define KIN_IK_STAMP(k)                                   \
    do {                                                  \
        const uint64_t t_ = ik_stamp();                   \
        if ((k) == KINHIP_IK_SECT) sect_acc += t_ - sect_prev; \
        sect_prev = t_;                                   \
    } while (0)
#else
#define KIN_IK_STAMP(k) \
    do {                \
    } while (0)
#endif

#if KINHIP_IK_NARROW
#define KIN_IK_LD ldn_soa
#define KIN_IK_ST stn_soa
#else
#define KIN_IK_LD ld_soa
#define KIN_IK_ST st_soa
#endif

// --------------------------------------------------------------------------
// shared phase-A evaluator for the IK kernels: q per step in registers
// --------------------------------------------------------------------------
template <typename T, int MAXA>
__device__ __forceinline__ void chain_records(const KProg<T>& P, const KStep<T>* __restrict__ S,
                                              const Fr<T>& root, const T (&qs)[MAXA], Fr<T>& L,
                                              T (&ro)[MAXA][3], T (&rz)[MAXA][3]) {
    Fr<T> f = root;
#pragma unroll
    for (int s = 0; s < MAXA; ++s) step_a<T, true>(f, S[s], qs[s], ro[s], rz[s]);  // fast trig (fp32)
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

// jcol with the linear part z x (p - o) already formed (ik_body computes it once per
// iteration into the record's origin slot: o := z x (p - o))
template <typename T, int ROWS>
__device__ __forceinline__ void jcol_pre(const KStep<T>& st, const T (&lin)[3], const T (&z)[3], T (&J)[ROWS]) {
    const T m = (st.flags & SF_REC) ? T(1) : T(0);
    if (st.jkind == MOT_PRISM) {
        J[0] = m * z[0]; J[1] = m * z[1]; J[2] = m * z[2];
        if constexpr (ROWS == 6) { J[3] = T(0); J[4] = T(0); J[5] = T(0); }
    } else {
        J[0] = m * lin[0]; J[1] = m * lin[1]; J[2] = m * lin[2];
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
    const T s = sqrt_fast(v0 * v0 + v1 * v1 + v2 * v2);
    const T c = T(0.5) * (E[0] + E[4] + E[8] - T(1));
#if KINHIP_IK_FAST_ATAN
    const T th = atan2_pos_fast(s, c);  // fp32: polynomial, 3.1e-7 abs (kinhip_device.h)
#else
    const T th = atan2_t(s, c);
#endif
    // common cases without a branch: k = th / s, or 1 for s <= 1e-7 (w = v exactly); only the
    // rotation by ~pi (s tiny, c < 0) takes the branch
    const bool tiny = !(s > T(1e-7));
    T kth;
    if constexpr (sizeof(T) == 4) kth = th * rcp_fast(s);
    else kth = th / s;
    kth = tiny ? T(1) : kth;
    w[0] = v0 * kth; w[1] = v1 * kth; w[2] = v2 * kth;
    if (tiny & !(c > T(0))) {
        int b = 0;
        if (E[4] > E[0]) b = 1;
        if (E[8] > E[4 * b]) b = 2;
        T a[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) a[k] = T(0.25) * (E[3 * k + b] + E[3 * b + k]);  // u_k u_b (E = 2uu^T - I)
        a[b] = T(0.5) * (E[4 * b] + T(1));                                            // u_b^2
        const T nn = sqrt_t(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
#pragma unroll
        for (int k = 0; k < 3; ++k) w[k] = a[k] / nn * th;
    }
}

template <bool F32>
struct ik_solve_type {
    using type = double;
};
template <>
struct ik_solve_type<true> {
    using type = float;
};

template <typename T>
struct IkArgsT {
    int32_t max_iters;
    T lam2, tol_pos, tol_rot, max_step;
    int32_t attempt_len;  // 0: no restarts
    int32_t n_attempts;   // 1 + (max_iters - 1) / attempt_len (attempts the sequential schedule reaches)
    uint64_t seed;
    int64_t ibase;  // global index of this chunk's first configuration
    // Two-phase schedule (launch_ik_dls, small batches): phase 1 runs attempt 0 of every target
    // (one lane each) and appends the targets it does not solve to fail_list instead of writing
    // them; phase 2 runs attempts att0 = 1, 2, ... of the listed targets only (idx = fail_list).
    // Otherwise att0 = 0, phase1 = 0, idx = null.
    // fail_list holds kIkSubRings rings of fail_mask + 1 entries (phase-1 wave w appends to ring
    // w % kIkSubRings, so the returning atomics of a launch spread over as many L2 lines instead of
    // queueing on one: ~6 us for 1,024 waves on one head).  Each ring has three control words on a
    // line of its own (fail_ctl + r * kIkCtlStride) that are never reset between calls (so no memset
    // launch precedes phase 1, and a captured graph replays as is): [0] = ring head (phase 1 appends
    // at atomicAdd(head) & mask), [1] = this call's first entry (phase 1 copies it from [2]), [2] =
    // the next call's first entry (phase 2 sets it to the head, after every phase-1 append).  Phase
    // 2's targets are the rings' entries [[1], [0]) in ring order (a prefix sum over the rings).
    int32_t att0;
    int32_t phase1;
    const int32_t* idx;
    int32_t* fail_list;
    uint32_t* fail_ctl;
    uint32_t fail_mask;
    // starting angles (kin_ik_dls_batch_from): read from q0 (same leading dimension as q) instead of
    // q, so q is written without being read and a caller keeps q0 for the next batch; null: q in place
    const T* q0;
    // 1: the reference's objective (kin_ik_params.with_rot = 2, src/inverse_kinematics.jl:38-50):
    // residual [p* - p; rpy* - rpy] (angle differences wrapped to (-pi, pi]) with the rpy_jac=true
    // Jacobian rows, converged on |dp| < tol_pos and |d rpy| < tol_rot; 0: the axis-angle residual
    int32_t rpy_obj;
    // Early hand-over (two-phase schedule): phase 1 stops attempt 0 of a target that is not solved
    // after p1_cut iterations (0: runs the whole attempt) and lists it with its state -- the angles
    // in q (and base in q's base columns), the active set in fail_aux at the same ring position;
    // phase 2 (cont = 1, att0 = 0) resumes attempt 0 there on slot 0 beside attempts 1, 2, ...
    // The resumed trajectory is the uninterrupted one bit for bit (nothing else carries over).
    int32_t p1_cut;
    int32_t cont;
    int32_t* fail_aux;
    // error-scaled damping (kin_ik_params.damp_err): the solve's lambda^2 + damp_err (|dp|^2 + |rot|^2)
    T damp_err;
    // phase 2 (> 0): list entries go to the first wave of each of the first p2_spread workgroups (the
    // workgroups the chip holds at once), then the second wave of each, ...: a short list spreads over all
    // CUs instead of filling the first workgroups' CUs two waves per SIMD, and never reaches past the
    // resident workgroups while it has fewer waves than they hold.  0: block-major waves.
    int32_t p2_spread;
    // kin_ik_dls_batch_trace: |dp| and |rot| of every iterate (rows 2 it, 2 it + 1 of [2 (max_iters + 1)]
    // [trace_ld]), or null
    T* trace;
    int64_t trace_ld;
    // k_ik_tree (kin_ik_coll_batch_alt): the restart origin -- attempt 1's free variables, every restart's base --
    // or null
    const T* q_alt;
};

// the objective inside ik_body: RPY < 0 reads it from the launch (IkArgsT::rpy_obj, the generic kernels); the
// specialised kernels compile it in (RPY = 0 axis-angle or position, 1 the reference's rpy objective): the
// iteration then carries neither the other objective's code nor the register copies that join the two paths
// (config 4: 0.072-0.075 -> 0.068-0.070 ms, identical results; profiles/r06_ik_rpy_const_ab.txt)
#define KIN_RPY(a) (RPY < 0 ? (a).rpy_obj != 0 : RPY != 0)
// lambda^2 + mu (ep^2 + er^2) rounded operation by operation, as the oracle forms it (no contraction)
template <typename S>
__device__ __forceinline__ S ik_damping(S lam2, S mu, S ep, S er) {
#pragma clang fp contract(off)
    return lam2 + mu * (ep * ep + er * er);
}

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
        T v;
        if (att > 0 && c >= 0 && (st.flags & SF_REC)) {
            // a restart draws the column: no load of q0 (a load here would wait, through
            // s_waitcnt vmcnt, for every store the wave still has in flight)
            double lo = (double)st.lo, hi = (double)st.hi;
            if (!isfinite(lo) || !isfinite(hi)) { lo = -3.14159265358979323846; hi = 3.14159265358979323846; }
            v = (T)(lo + (hi - lo) * ik_seed_u01(a.seed, gi, att, c));
        } else {
            v = c >= 0 ? KIN_IK_LD(q, c, ldq, off) : T(0);
            if (att > 0 && c >= 0) v = fmin(fmax(v, st.lo), st.hi);  // attempt 0's first step has clamped it
        }
        qs[s] = v;
    }
}

// inclusive prefix sum over the 64 lanes by DPP adds (row_shr 1, 2, 4, 8 inside each 16-lane row, then
// row_bcast 15 / 31 across rows): six VALU instructions instead of six dependent ds_bpermute round trips
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    int t = (int)v;
    t += __builtin_amdgcn_update_dpp(0, t, 0x111, 0xF, 0xF, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x112, 0xF, 0xF, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x114, 0xF, 0xF, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x118, 0xF, 0xF, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x142, 0xA, 0xF, false);
    t += __builtin_amdgcn_update_dpp(0, t, 0x143, 0xC, 0xF, false);
    return (uint32_t)t;
}

// min over the G lanes of an aligned lane group by DPP moves (quad_perm [1,0,3,2], [2,3,0,1], then
// row_half_mirror for 8-lane groups): VALU only, where __shfl_xor compiles to ds_bpermute, an LDS round
// trip of ~100 cycles each, two per IK iteration at G = 4, in series, at one wave per SIMD
template <int G>
__device__ __forceinline__ int group_min(int v) {
    if constexpr (G > 8) {
#pragma unroll
        for (int w = 1; w < G; w <<= 1) v = min(v, __shfl_xor(v, w, G));
    } else {
        if constexpr (G >= 2) v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));
        if constexpr (G >= 4) v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));
        if constexpr (G >= 8) v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false));
    }
    return v;
}

// Work distribution: wave w owns targets [w*chunk, (w+1)*chunk) and keeps its
// 64/G lane groups busy: a group whose target is finished (all its lanes done)
// writes the result and takes the wave's next target at once, so a wave no
// longer waits for its slowest target before the others move on.  The queue is
// wave-local (ballot + popcount, no atomics, nothing in memory between launches).
template <typename T, int MAXA, int ROWS, int G, int RPY = -1, bool F64S = true>
__device__ __forceinline__ void ik_body(const KProg<T>& P, const KStep<T>* __restrict__ S, const IkArgsT<T>& a,
                                        const T* __restrict__ tgt, int64_t ldt, T* __restrict__ q, int64_t ldq,
                                        int64_t n, int32_t* __restrict__ iters, T* __restrict__ err, int64_t lde,
                                        int64_t chunk) {
    const int lane = (int)(threadIdx.x & 63u);
    const int slot = lane % G, grp = lane / G;
    int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (a.idx && a.p2_spread > 0) {  // rounds of p2_spread workgroups of 4 waves, wave slot-major in a round
        const uint32_t R = (uint32_t)a.p2_spread, b = blockIdx.x, r0 = b / R * R;
        const uint32_t rr = gridDim.x - r0 < R ? gridDim.x - r0 : R;
        wave = (int64_t)r0 * 4 + (int64_t)(threadIdx.x >> 6) * rr + (b - r0);
    }
    // two-phase control words (see IkArgsT): one lane per ring of the grid's first wave moves its start marks
    if (blockIdx.x == 0 && threadIdx.x < (unsigned)kIkSubRings && (a.phase1 || a.idx)) {
        uint32_t* c = a.fail_ctl + threadIdx.x * kIkCtlStride;
        if (a.phase1) c[1] = c[2];
        else c[2] = c[0];
    }
    // phase 2: lane r of every wave holds ring r's first entry and the number of listed targets
    // before ring r (exclusive prefix over the rings); the wave's share is entries of that order
    uint32_t ring_beg = 0, ring_excl = 0;
    int64_t nt = n;
    static_assert(kIkSubRings == 64, "one ring per lane of the phase-2 prefix");
    if (a.idx) {  // (uniform)
        const uint32_t* c = a.fail_ctl + lane * kIkCtlStride;
        ring_beg = c[1];
        const uint32_t cnt = c[0] - ring_beg;
        const uint32_t inc = wave_incl_scan(cnt);
        ring_excl = inc - cnt;
        nt = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)inc, 63);  // phase 2: the listed targets only
    }
    const T* __restrict__ qin = a.q0 ? a.q0 : q;  // uniform: where the starting angles are read
    const int64_t wbeg = wave * chunk, wend = wbeg + chunk < nt ? wbeg + chunk : nt;
    int64_t next = wbeg;  // wave-uniform: next unassigned target of this wave
    int64_t i = 0;
    uint32_t rpos = 0;    // phase 2: ring position of this target (fail_aux)
    bool have = false;    // the first pass of the loop hands every group its first target
    const bool base = (P.flags & PF_BASE) != 0;
    const int L = a.attempt_len;
    const uint64_t gmask = (G == 64) ? ~0ull : (((1ull << G) - 1ull) << (grp * G));

    T Rt[9], pt[3], b0[3], qs[MAXA], b[3];
    T trpy[3] = {T(0), T(0), T(0)};  // rpy of the target (reference objective)
    uint32_t blk = 0;  // active set: joints held out of the solve (bit s = phase-A step s)
    int att = 0, it = 0, res_att = INT_MAX;
    int att_end = INT_MAX;  // iteration at which this lane's attempt is over (the schedule's it % L == 0)
    bool done = true, final_lane = false;
    uint32_t off = 0;
    T ep = 0, er = 0;
#if KINHIP_IK_SECT
    uint64_t sect_acc = 0, sect_prev = 0, sect_t0 = 0;
    // KINHIP_IK_SECT=9: the lane's entry and write times (s_memrealtime, 100 MHz, low 32 bits as raw
    // bits in err rows 0 / 1) to place each launch's waves on one clock
    const uint32_t rt_entry = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
    auto start_target = [&]() {
        off = (uint32_t)i * (uint32_t)sizeof(T);
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int c = 0; c < 3; ++c) Rt[3 * r + c] = KIN_IK_LD(tgt, r + 3 * c, ldt, off);
            pt[r] = KIN_IK_LD(tgt, 9 + r, ldt, off);
        }
        if (ROWS == 6 && KIN_RPY(a)) {
            T kk[6];
            rpy_and_rate<KINHIP_IK_FAST_ATAN != 0>(Rt, trpy, kk);
        }
        b0[0] = b0[1] = b0[2] = T(0);
        if (base)
            for (int k = 0; k < 3; ++k) b0[k] = KIN_IK_LD(qin, P.base_col + k, ldq, off);
        b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2];
        att = a.att0 + slot;
        done = att >= a.n_attempts;
        res_att = INT_MAX;
        final_lane = false;
        it = att > 0 ? att * L + 1 : 0;
        ep = er = T(0);
        blk = 0;
        att_end = L > 0 ? (att + 1) * L : INT_MAX;
        if (a.phase1 && a.p1_cut) att_end = a.p1_cut;  // phase 1: attempt 0 only, handed over there
        if (a.cont && att == 0) {  // resume attempt 0 where phase 1 handed it over
            it = a.p1_cut;
            blk = (uint32_t)a.fail_aux[rpos];
#pragma unroll
            for (int s = 0; s < MAXA; ++s) {
                const int32_t c = S[s].qcol;
                qs[s] = c >= 0 ? KIN_IK_LD(q, c, ldq, off) : T(0);
            }
            if (base)
                for (int k = 0; k < 3; ++k) b[k] = KIN_IK_LD(q, P.base_col + k, ldq, off);
        } else {
            ik_start_attempt<T, MAXA>(S, a, qin, ldq, off, a.ibase + i, att, qs);
        }
    };
    T ro[MAXA][3], rz[MAXA][3];
    for (;;) {
        int gm = res_att;  // lowest converged attempt of this lane group's target so far
        if constexpr (G > 1) {
            gm = group_min<G>(gm);  // (every lane of the wave is here: the loop only exits wave-wide)
            if (have && !done && gm < att) done = true;
        }
        // a group whose lanes are all done writes its target and takes the next one
        // While the wave's range still has targets, a finished group writes at once and takes the next;
        // once every target is handed out (always, for a wave of at most 64 / G targets) the finished
        // groups keep their results in registers and the whole wave writes when its last lane is
        // done: no stores and no bookkeeping inside the iterations
        const uint64_t dmask = __ballot(!have || done);
        if (next >= wend ? dmask == ~0ull : dmask != 0ull) {  // (wave-uniform)
        const bool gfin = have && (dmask & gmask) == gmask;
        // attempt 0 failed or was handed over: phase 2 takes the target.  The ring positions of the
        // wave's hand-overs come first, from one returning atomic issued by one lane: its wait then
        // covers none of this pass's result stores (which it did when placed after them)
        const bool handover = gfin && a.phase1 && res_att == INT_MAX;
        uint32_t pos = 0;
        if (a.phase1) {  // (uniform)
            const uint64_t hmask = __ballot(handover);
            if (hmask) {  // (uniform)
                const int lead = __ffsll((unsigned long long)hmask) - 1;
                uint32_t first = 0;
                const uint32_t ring = (uint32_t)(wave % kIkSubRings);
                if (lane == lead) first = atomicAdd(a.fail_ctl + ring * kIkCtlStride, (uint32_t)__popcll(hmask));
                first = __shfl(first, lead);
                pos = ring * (a.fail_mask + 1u) +
                      ((first + (uint32_t)__popcll(hmask & ((1ull << lane) - 1ull))) & a.fail_mask);
            }
        }
        if (gfin) {
            const bool writer = (G > 1) ? ((gm != INT_MAX) ? (res_att == gm) : final_lane) : true;
            if (handover) {
                a.fail_list[pos] = (int32_t)i;
                if (a.p1_cut) {  // hand-over state (see IkArgsT)
                    a.fail_aux[pos] = (int32_t)blk;
#pragma unroll
                    for (int s2 = 0; s2 < MAXA; ++s2) {
                        const int32_t c = S[s2].qcol;
                        if (c >= 0) KIN_IK_ST(q, c, ldq, off, qs[s2]);
                    }
                    if (base)
                        for (int k = 0; k < 3; ++k) KIN_IK_ST(q, P.base_col + k, ldq, off, b[k]);
                }
            } else if (writer) {
#pragma unroll
                for (int s2 = 0; s2 < MAXA; ++s2) {
                    const int32_t c = S[s2].qcol;
                    if (c >= 0) KIN_IK_ST(q, c, ldq, off, qs[s2]);
                }
                if (base)
                    for (int k = 0; k < 3; ++k) KIN_IK_ST(q, P.base_col + k, ldq, off, b[k]);
                if (iters) iters[i] = it;
#if KINHIP_IK_SECT == 9
                if constexpr (sizeof(T) == 4) {
                    ep = __uint_as_float(rt_entry);
                    er = __uint_as_float((uint32_t)__builtin_amdgcn_s_memrealtime());
                }
#elif KINHIP_IK_SECT
                ep = (T)(double)sect_acc;
                er = (T)(double)(ik_stamp() - sect_t0);
#endif
                if (err) {
                    KIN_IK_ST(err, 0, lde, off, ep);
                    KIN_IK_ST(err, 1, lde, off, er);
                }
            }
            have = false;
        }
        const uint64_t need = __ballot(!have && slot == 0) & ~0ull;  // group leaders asking for work
        if (need && next < wend) {
            const uint64_t lead = 1ull << (grp * G);
            const int rank = __popcll(need & (lead - 1ull));
            if (a.idx) {  // (uniform) phase 2: entry e = next + rank -> its ring (the last ring starting at or
                // before e).  The wave's entries [e0, e1] span few rings: a uniform binary search (v_readlane)
                // finds the ring of e0, then the lanes step over the rings that start inside (e0, e1]
                const uint32_t e = (uint32_t)(next + rank);
                const uint32_t e0 = (uint32_t)next, e1 = (uint32_t)next + (uint32_t)__popcll(need) - 1u;
                int r0 = 0;
#pragma unroll
                for (int step = kIkSubRings / 2; step >= 1; step >>= 1)
                    if ((uint32_t)__builtin_amdgcn_readlane((int)ring_excl, r0 + step) <= e0) r0 += step;
                uint32_t rb = (uint32_t)__builtin_amdgcn_readlane((int)ring_beg, r0);
                uint32_t rx = (uint32_t)__builtin_amdgcn_readlane((int)ring_excl, r0);
                int r = r0;
                for (int rr = r0 + 1; rr < kIkSubRings; ++rr) {
                    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)ring_excl, rr);
                    if (x > e1) break;  // (uniform)
                    if (x <= e) {
                        r = rr;
                        rx = x;
                        rb = (uint32_t)__builtin_amdgcn_readlane((int)ring_beg, rr);
                    }
                }
                rpos = (uint32_t)r * (a.fail_mask + 1u) + ((rb + (e - rx)) & a.fail_mask);
            }
            if (!have && (need & lead) && next + rank < wend) {
                i = a.idx ? (int64_t)a.idx[rpos] : next + rank;
                have = true;
                start_target();  // the single (inlined) initialisation site
            }
            next += __popcll(need);
        }
        if (__ballot(have) == 0) break;  // wave-uniform exit: range drained, every target written
        }
        if (!have || done) continue;
#if KINHIP_IK_SECT
        if (sect_t0 == 0) sect_t0 = sect_prev = ik_stamp();
#endif
        KIN_IK_STAMP(7);
        Fr<T> root, L_;
        if (base) base_frame(root, b[0], b[1], b[2]);
        else set_identity(root);
        chain_records<T, MAXA>(P, S, root, qs, L_, ro, rz);
        KIN_IK_STAMP(1);
        const Fr<T>& Lf = L_;
        T e[6];
        e[0] = pt[0] - Lf.t[0]; e[1] = pt[1] - Lf.t[1]; e[2] = pt[2] - Lf.t[2];
        ep = sqrt_fast(e[0] * e[0] + e[1] * e[1] + e[2] * e[2]);
        er = T(0);
        T kr[6];  // rpy_derivative! coefficients (reference objective)
        if constexpr (ROWS == 6) {
            T w[3];
            if (KIN_RPY(a)) {  // wave-uniform
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
        if (a.trace) {  // (uniform) kin_ik_dls_batch_trace: this iterate's residual norms
            st_soa(a.trace, 2 * (int64_t)it, a.trace_ld, off, ep);
            st_soa(a.trace, 2 * (int64_t)it + 1, a.trace_ld, off, er);
        }
        // the rare ends of an iteration behind one branch (bitwise, so the common path carries no
        // exec-mask bookkeeping): converged, out of iterations (only the last attempt gets there),
        // attempt over (phase 1 with a hand-over: the target goes to phase 2)
        const bool conv = (ep < a.tol_pos) & (er < a.tol_rot);
        if (conv | (it >= a.max_iters) | (it == att_end)) {
            if (conv) {
                res_att = att;
                done = true;
            } else if (it >= a.max_iters) {
                final_lane = true;
                it = a.max_iters + 1;  // not converged (kinhip.h: iters > max_iters)
                done = true;
            } else {  // attempt over: this lane's next one, if any
                att += G;
                if (att >= a.n_attempts) {
                    done = true;
                } else {
                    it = att * L + 1;
                    att_end = (att + 1) * L;
                    ik_start_attempt<T, MAXA>(S, a, qin, ldq, off, a.ibase + i, att, qs);
                    b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2];
                    blk = 0;
                }
            }
            continue;
        }

        KIN_IK_STAMP(2);
        // linear Jacobian rows z x (p - o) once per iteration (the solve and dq reuse them)
#pragma unroll
        for (int s = 0; s < MAXA; ++s) {
            if (S[s].jkind == MOT_PRISM) continue;  // [z; 0] (jcol_pre): no lever arm
            const T dx = Lf.t[0] - ro[s][0], dy = Lf.t[1] - ro[s][1], dz = Lf.t[2] - ro[s][2];
            ro[s][0] = fma(rz[s][1], dz, -(rz[s][2] * dy));
            ro[s][1] = fma(rz[s][2], dx, -(rz[s][0] * dz));
            ro[s][2] = fma(rz[s][0], dy, -(rz[s][1] * dx));
        }
        if constexpr (ROWS == 6) {
            if (KIN_RPY(a)) {  // angular rows -> d(rpy)/dq (get_jacobian!(...; rpy_jac=true))
#pragma unroll
                for (int s = 0; s < MAXA; ++s) {
                    if (S[s].jkind == MOT_PRISM) continue;  // [z; 0]: its linear part is z itself
                    const T x = rz[s][0], y = rz[s][1], z = rz[s][2];
                    rz[s][0] = fma(kr[0], x, kr[1] * y);
                    rz[s][1] = fma(kr[2], x, kr[3] * y);
                    rz[s][2] = fma(kr[4], x, fma(kr[5], y, z));
                }
            }
        }
        // Active set (same rule as the oracle's or_ik_dls_batch): a joint that sits on a limit and
        // that the previous iteration's unconstrained direction pushed further out is held out of
        // this solve (weight 0); it rejoins once the direction J_s^T y points back inside.  One
        // solve per iteration: the set lags one iteration instead of re-solving in the same one
        // (the re-solve ran in ~half of all lane-iterations, i.e. in nearly every wave-iteration).
        T dq[MAXA], db[3] = {T(0), T(0), T(0)};
        T mx = T(0);
        // the damped solve in arithmetic type TS: fp64 (also in the fp32 kernel, KINHIP_IK_F64SOLVE)
        auto damped_solve = [&](auto ts_tag) {
            using TS = decltype(ts_tag);
            constexpr bool refine = sizeof(T) == 4 && KINHIP_IK_F64SOLVE == 2;
            using YS = typename ik_solve_type<!refine && sizeof(TS) == 4>::type;  // type of the solution y
            TS Jb[3][ROWS];
            if (base) {
#pragma unroll
                for (int k = 0; k < 3; ++k)
#pragma unroll
                    for (int r = 0; r < ROWS; ++r) Jb[k][r] = TS(0);
                Jb[0][0] = TS(1);
                Jb[1][1] = TS(1);
                Jb[2][0] = -(TS)(Lf.t[1] - b[1]);
                Jb[2][1] = (TS)(Lf.t[0] - b[0]);
                if constexpr (ROWS == 6) Jb[2][5] = TS(1);
            }
            // A = J W J^T + lambda^2 I  (lower triangle)
            TS A[ROWS][ROWS];
            // (damp_err is uniform: a fixed-lambda call runs no extra instructions)
            const TS lam2 = a.damp_err != T(0) ? ik_damping<TS>((TS)a.lam2, (TS)a.damp_err, (TS)ep, (TS)er)
                                               : (TS)a.lam2;
#pragma unroll
            for (int r = 0; r < ROWS; ++r)
#pragma unroll
                for (int c = 0; c < ROWS; ++c) A[r][c] = (r == c) ? lam2 : TS(0);
            // fp32 solve: entries (r, 2k) and (r, 2k + 1) in one packed FMA (v_pk_fma_f32, J[r] broadcast):
            // 12 instead of 21 per joint, each element the same fma (identical results).  One wave per
            // SIMD issues a packed FMA in ~1.5x the time of a scalar one (tools/pk_probe.hip).
            constexpr bool pk = KINHIP_IK_PK && sizeof(TS) == 4 && ROWS == 6;
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 A2[pk ? ROWS : 1][pk ? ROWS / 2 : 1];
            if constexpr (pk) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r)
#pragma unroll
                    for (int k = 0; k < ROWS / 2; ++k) A2[r][k] = f2{(float)A[r][2 * k], (float)A[r][2 * k + 1]};
            }
#pragma unroll
            for (int s = 0; s < MAXA; ++s) {
                T J[ROWS];
                jcol_pre<T, ROWS>(S[s], ro[s], rz[s], J);
                const bool wt = (S[s].flags & SF_REC) && S[s].qcol >= 0;  // (a constant in specialised kernels)
                const T ws = wt && ((blk >> s) & 1u) ? T(0) : T(1);
                if (wt && !pk) {
#pragma unroll
                    for (int r = 0; r < ROWS; ++r) J[r] *= ws;
                }
                const int nr = (ROWS == 6 && S[s].jkind == MOT_PRISM) ? 3 : ROWS;  // prismatic: linear block only
                if constexpr (pk) {
                    // the weight on the pair operand only (3 packed multiplies instead of 6): fma(J_r, ws J_c, a)
                    // equals fma(ws J_r, ws J_c, a) for ws in {0, 1} (a held column adds an exact zero; the sums
                    // are never -0), so every kernel variant keeps identical results
                    f2 Jp[3] = {f2{(float)J[0], (float)J[1]}, f2{(float)J[2], (float)J[3]},
                                f2{(float)J[4], (float)J[5]}};
                    if (wt) {
#pragma unroll
                        for (int k = 0; k < 3; ++k) Jp[k] = Jp[k] * f2{(float)ws, (float)ws};
                    }
#pragma unroll
                    for (int r = 0; r < ROWS; ++r)
#pragma unroll
                        for (int k = 0; k <= r / 2; ++k)
                            if (r < nr && 2 * k < nr)
                                A2[r][k] = __builtin_elementwise_fma(f2{(float)J[r], (float)J[r]}, Jp[k], A2[r][k]);
                } else {
#pragma unroll
                    for (int r = 0; r < ROWS; ++r)
#pragma unroll
                        for (int c = 0; c <= r; ++c)
                            if (r < nr) A[r][c] = fma((TS)J[r], (TS)J[c], A[r][c]);
                }
            }
            if constexpr (pk) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r)
#pragma unroll
                    for (int c = 0; c <= r; ++c) A[r][c] = (TS)((c & 1) ? A2[r][c / 2].y : A2[r][c / 2].x);
            }
            if (base) {
#pragma unroll
                for (int k = 0; k < 3; ++k)
#pragma unroll
                    for (int r = 0; r < ROWS; ++r)
#pragma unroll
                        for (int c = 0; c <= r; ++c) A[r][c] = fma(Jb[k][r], Jb[k][c], A[r][c]);
            }
            KIN_IK_STAMP(3);
            // Cholesky A = L L^T (in place, lower), then y = A^-1 e.  The fp32 kernel keeps the
            // reciprocal square root of each pivot and multiplies: the 6 square roots and 27 divisions
            // of the IEEE form are ~10 instructions each and dominated the iteration -- v_rsq_f32 for an
            // fp32 solve, v_rsq_f64 plus one Newton step (~2^-44) for its fp64 solve.  The fp64 kernel
            // takes the IEEE square root and one IEEE reciprocal per pivot, which multiplies (6 divisions
            // instead of 27; the oracle's chol_solve, iterates compared with or_ik_dls_batch to 1e-7).
            constexpr bool fast = sizeof(T) == 4;
            auto rsq = [](TS d) -> TS {
                if constexpr (sizeof(TS) == 4) {
                    return rsqrt_fast(d);
                } else {
                    const double r = __builtin_amdgcn_rsq(d);
                    return r * fma(-0.5 * d * r, r, 1.5);
                }
            };
            TS ip[ROWS];  // 1 / L[j][j] (fp32 kernel)
#pragma unroll
            for (int j = 0; j < ROWS; ++j) {
                TS d = A[j][j];
#pragma unroll
                for (int k = 0; k < j; ++k) d = fma(-A[j][k], A[j][k], d);
                if constexpr (fast) {
                    ip[j] = rsq(d);
                } else {
                    d = sqrt_t(d);
                    A[j][j] = d;
                    ip[j] = TS(1) / d;
                }
#pragma unroll
                for (int r = j + 1; r < ROWS; ++r) {
                    TS sm = A[r][j];
#pragma unroll
                    for (int k = 0; k < j; ++k) sm = fma(-A[r][k], A[j][k], sm);
                    A[r][j] = sm * ip[j];
                }
            }
            auto chol_solve = [&](const TS (&rhs)[ROWS], TS (&x)[ROWS]) {
#pragma unroll
                for (int r = 0; r < ROWS; ++r) {
                    TS sm = rhs[r];
#pragma unroll
                    for (int k = 0; k < r; ++k) sm = fma(-A[r][k], x[k], sm);
                    x[r] = sm * ip[r];
                }
#pragma unroll
                for (int r = ROWS - 1; r >= 0; --r) {
                    TS sm = x[r];
#pragma unroll
                    for (int k = r + 1; k < ROWS; ++k) sm = fma(-A[k][r], x[k], sm);
                    x[r] = sm * ip[r];
                }
            };
            TS e_s[ROWS], y0[ROWS];
#pragma unroll
            for (int r = 0; r < ROWS; ++r) e_s[r] = (TS)e[r];
            chol_solve(e_s, y0);
            YS y[ROWS];
#pragma unroll
            for (int r = 0; r < ROWS; ++r) y[r] = (YS)y0[r];
            if constexpr (refine) {
                // r = e - lambda'^2 y - J W (J^T y) - Jb Jb^T y in fp64, from the weighted columns of A
                double res[ROWS];
#pragma unroll
                for (int r = 0; r < ROWS; ++r) res[r] = fma(-(double)lam2, y[r], (double)e[r]);
#pragma unroll
                for (int s = 0; s < MAXA; ++s) {
                    T J[ROWS];
                    jcol_pre<T, ROWS>(S[s], ro[s], rz[s], J);
                    if ((S[s].flags & SF_REC) && S[s].qcol >= 0 && ((blk >> s) & 1u)) continue;  // held: W = 0
                    const int nr = (ROWS == 6 && S[s].jkind == MOT_PRISM) ? 3 : ROWS;
                    double u = 0.0;
#pragma unroll
                    for (int r = 0; r < ROWS; ++r)
                        if (r < nr) u = fma((double)J[r], y[r], u);
#pragma unroll
                    for (int r = 0; r < ROWS; ++r)
                        if (r < nr) res[r] = fma(-(double)J[r], u, res[r]);
                }
                if (base) {
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        double u = 0.0;
#pragma unroll
                        for (int r = 0; r < ROWS; ++r) u = fma((double)Jb[k][r], y[r], u);
#pragma unroll
                        for (int r = 0; r < ROWS; ++r) res[r] = fma(-(double)Jb[k][r], u, res[r]);
                    }
                }
                TS rs[ROWS], dl[ROWS];
#pragma unroll
                for (int r = 0; r < ROWS; ++r) rs[r] = (TS)res[r];
                chol_solve(rs, dl);
#pragma unroll
                for (int r = 0; r < ROWS; ++r) y[r] = y[r] + (YS)dl[r];
            }
            KIN_IK_STAMP(4);
            uint32_t nb = 0;
#pragma unroll
            for (int s = 0; s < MAXA; ++s) {
                T J[ROWS];
                jcol_pre<T, ROWS>(S[s], ro[s], rz[s], J);
                YS vs = YS(0);
                const int nr = (ROWS == 6 && S[s].jkind == MOT_PRISM) ? 3 : ROWS;  // (zero angular rows)
#pragma unroll
                for (int r = 0; r < ROWS; ++r)
                    if (r < nr) vs = fma((YS)J[r], y[r], vs);
                const T v = (T)vs;
                const bool held = (blk >> s) & 1u;
                dq[s] = held ? T(0) : v;
                // pushed further out of a limit it sits on (selects, no short-circuit branches)
                const T out_lo = qs[s] <= S[s].lo ? -v : T(0), out_hi = qs[s] >= S[s].hi ? v : T(0);
                nb |= ((out_lo > T(0)) | (out_hi > T(0))) ? 1u << s : 0u;
                mx = fmax(mx, fabs(dq[s]));
            }
            blk = nb;
            if (base) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    YS v = YS(0);
#pragma unroll
                    for (int r = 0; r < ROWS; ++r) v = fma((YS)Jb[k][r], y[r], v);
                    db[k] = (T)v;
                    mx = fmax(mx, fabs(db[k]));
                }
            }
        };
        if constexpr (sizeof(T) == 4 && KINHIP_IK_F64SOLVE == 3) {
            // fp64 for the first iterations of attempt 0 (the caller's q0), fp32 elsewhere (see the macro).  F64S =
            // false: a launch where that never holds (phase 2 of the two-phase schedule with a hand-over point of at
            // least KINHIP_IK_F64_ITERS and lambda^2 >= KINHIP_IK_F32SOLVE_MIN_LAM2; launch_ik_dls) compiles the fp64
            // solve out -- the same arithmetic, without its code and registers in the loop
            if (F64S && ((att == 0 && it < KINHIP_IK_F64_ITERS) || a.lam2 < T(KINHIP_IK_F32SOLVE_MIN_LAM2)))
                damped_solve(double());
            else
                damped_solve(float());
        } else {
            damped_solve(typename ik_solve_type<sizeof(T) == 4 && KINHIP_IK_F64SOLVE != 1>::type());
        }
        KIN_IK_STAMP(5);
        const T sc = mx > a.max_step ? a.max_step / mx : T(1);
#pragma unroll
        for (int s = 0; s < MAXA; ++s) qs[s] = fmin(fmax(fma(sc, dq[s], qs[s]), S[s].lo), S[s].hi);
        if (base)
            for (int k = 0; k < 3; ++k) b[k] = fma(sc, db[k], b[k]);
        ++it;
        KIN_IK_STAMP(6);
    }
}

// --------------------------------------------------------------------------
// k_nakamura: point_inverse_kinematics_nakamura, 50 iterations
// --------------------------------------------------------------------------
template <typename T, int MAXA>
__device__ __forceinline__ void nakamura_body(const KProg<T>& P, const KStep<T>* __restrict__ S,
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

}  // namespace
}  // namespace kinhip

#pragma clang fp contract(fast)  // (the translation unit's default again: -ffp-contract=fast-honor-pragmas)
