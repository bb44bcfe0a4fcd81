// kinhip_ik.hip -- k_ik_dls (batched DLS IK with restarts) and k_nakamura.
// (gfx950 only; shared helpers in kinhip_device.h)
#include "kinhip_ik_dev.h"

namespace kinhip {
namespace {

// --------------------------------------------------------------------------
// generic kernels (the staged program is read from device memory)
// --------------------------------------------------------------------------
#ifndef KINHIP_IK_WAVES
#define KINHIP_IK_WAVES 1
#endif
template <typename T, int MAXA, int ROWS, int G>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KINHIP_IK_WAVES))) void k_ik_dls(
    const KProg<T> P, const KStep<T>* __restrict__ S, const IkArgsT<T> a, const T* __restrict__ tgt, int64_t ldt,
    T* __restrict__ q, int64_t ldq, int64_t n, int32_t* __restrict__ iters, T* __restrict__ err, int64_t lde,
    int64_t chunk) {
    ik_body<T, MAXA, ROWS, G>(P, S, a, tgt, ldt, q, ldq, n, iters, err, lde, chunk);
}

template <typename T, int MAXA>
__global__ __launch_bounds__(256) void k_nakamura(const KProg<T> P, const KStep<T>* __restrict__ S,
                                                  const T* __restrict__ pts, int64_t ldpt, T* __restrict__ q,
                                                  int64_t ldq, int64_t n) {
    nakamura_body<T, MAXA>(P, S, pts, ldpt, q, ldq, n);
}

}  // namespace

// Lanes per IK target (parallel restart attempts): enough to put ~8 waves on
// every SIMD for small batches, never more than the attempts the schedule has.
// KINHIP_IK_GROUP=<1|2|4|8> overrides (A/B).
static int ik_group(int64_t n, int n_attempts, int lanes) {
    static const int env = ab_env_int("KINHIP_IK_GROUP", 0);
    const int forced = lanes ? lanes : env;
    if (forced == 1 || forced == 2 || forced == 4 || forced == 8) return forced;
    int g = 1;
    while (g < n_attempts && g < 8 && n * g * 2 <= (int64_t(1) << 19)) g *= 2;
    return g;
}

static int ik_cus() {
    static const int cus = [] {
        int dev = 0, c = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        return c > 0 ? c : 256;
    }();
    return cus;
}

// waves per CU that stay resident: 2 per SIMD for the generic kernels (~190-240 VGPRs);
// KINHIP_IK_RESIDENT=<waves per CU> overrides (A/B build only)
static int64_t ik_resident_waves() {
    static const int res_env = ab_env_int("KINHIP_IK_RESIDENT", 0);
    return (int64_t)ik_cus() * (res_env > 0 ? res_env : 8);
}

// Two-phase schedule (KINHIP_IK_TWO_PHASE=<0|1> in the A/B build, default automatic): a chunk of
// c targets runs in two phases when the caller left the lanes to the engine, there are restart
// attempts, the chunk fits the scratch ring and it needs more than one round of resident waves at
// the one-phase schedule's lanes per target.  kin_ik_dls_batch allocates the scratch only when
// this holds for some chunk of the call (n = the whole call, c = this chunk).
static bool ik_two_phase(const IkArgs& a, int64_t n, int64_t c, int64_t cap) {
    static const int tp_env = ab_env_int("KINHIP_IK_TWO_PHASE", -1);
    int L, natt;
    ik_attempts(a, &L, &natt);
    if (natt <= 1 || c > cap || a.lanes != 0) return false;
    const int64_t ng = 64 / ik_group(n, natt, a.lanes);
    const int64_t plain = (c + ng - 1) / ng;
    return tp_env >= 0 ? tp_env != 0 : plain > ik_resident_waves();
}

// Launch chunk of a call: kIkChunk (32-bit lane offsets), and with restarts at most the two-phase scratch
// capacity, so that a batch larger than one list still runs the two-phase schedule chunk by chunk (the chunks
// run in stream order on the call's scratch set; each target's arithmetic is unchanged).  2M targets: 1.20 ms
// on the one-phase queue before.
static int64_t ik_chunk(const IkArgs& a, int64_t cap) {
    int L, natt;
    ik_attempts(a, &L, &natt);
    return natt > 1 && a.lanes == 0 && cap > 0 ? std::min<int64_t>(kIkChunk, cap) : kIkChunk;
}

bool ik_wants_two_phase(const IkArgs& a, int64_t n, int64_t cap) {
    const int64_t chunk = ik_chunk(a, cap);
    for (int64_t s0 = 0; s0 < n; s0 += chunk)
        if (ik_two_phase(a, n, std::min<int64_t>(chunk, n - s0), cap)) return true;
    return false;
}

// Phase-1 hand-over point (IkArgsT::p1_cut): 5/8 of an attempt by default.  Config 4 (L = 16):
// 23% of the targets are still unsolved after 10 iterations (46% after 8, 4% after 16; oracle
// histogram), so phase 2 keeps about one wave per SIMD; measured 0.081 ms vs 0.089 (no hand-over),
// 0.092 (cut 8), 0.084 (cut 12) fp32 and 0.165 / 0.179 / 0.236 / 0.170 ms fp64
// (profiles/r03_ik_handover.txt).  With error-scaled damping (damp_err > 0) attempt 0 converges
// sooner (93% within 10 iterations), and half an attempt is the faster cut: config 4 damped 0.079 ms
// at cut 8 vs 0.088 at 10 (fixed lambda: 0.141 vs 0.082; profiles/r04_ik_p1_cut_ab.txt).
// KINHIP_IK_P1_CUT=<iterations> overrides (A/B build; 0 disables).
// 0 when the hand-over is not allowed or not shorter than L.
static int ik_p1_cut(int L, bool allowed, bool damped) {
    static const int env = ab_env_int("KINHIP_IK_P1_CUT", -1);
    const int cut = env >= 0 ? env : damped ? L / 2 : (5 * L) / 8;
    return allowed && cut > 0 && cut < L ? cut : 0;
}

thread_local bool g_ik_partial = false;
bool ik_last_call_partial() { return g_ik_partial; }

template <typename T>
hipError_t launch_ik_dls(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const IkArgs& a,
                         const T* target, int64_t ldt, const T* q0, T* q, int64_t ldq, int64_t n, int32_t* iters,
                         T* err, int64_t lde, const JitFns* jf, const IkScratch& scr, hipStream_t st) {
    int L, natt;
    ik_attempts(a, &L, &natt);
    g_ik_partial = false;
    IkArgsT<T> at{a.max_iters, T(a.lambda * a.lambda), T(a.tol_pos), T(a.tol_rot), T(a.max_step), L, natt, a.seed,
                  0, 0, 0, nullptr, nullptr, nullptr, 0u, nullptr, a.with_rot == 2 ? 1 : 0};
    at.damp_err = T(a.damp_err);
    at.trace = (T*)a.trace;
    at.trace_ld = a.trace_ld;
    const int G = ik_group(n, natt, a.lanes);
    const int cus = ik_cus();
    const int64_t resident_waves = ik_resident_waves();
    // queue depth: one target per group (no refill) while the batch fills the chip in at most
    // two rounds of waves, else as many waves as stay resident, each working through its share
    static const int qmode = ab_env_int("KINHIP_IK_QUEUE", -1);
    // Two-phase schedule (ik_two_phase): small batches fill the chip only by running the restart
    // attempts of a target side by side (G lanes), and a wave then lasts as long as any of its
    // targets' attempts.  Phase 1 runs attempt 0 of every target on one lane and writes the solved
    // ones; phase 2 runs attempts 1, 2, ... side by side for the ones attempt 0 did not solve, packed
    // densely (fail_list, a ring: IkArgsT).  Each attempt's arithmetic is unchanged and the lowest
    // converged attempt is still the one written: results are identical.
    // KINHIP_IK_TP_QUEUE=<0|1> (A/B): phase 1 of a large batch on wave-local queues; default:
    // automatic (only where the queue's resident waves do not lower the kernel's occupancy)
    static const int tpq_env = ab_env_int("KINHIP_IK_TP_QUEUE", -1);
    auto one = [&](IkArgsT<T>& ar, int GG, int64_t s0, int64_t c, int64_t per_wave, int64_t nw,
                   int bs = 256, bool no_f64 = false) -> hipError_t {
        const dim3 grid((unsigned)((nw * 64 + bs - 1) / bs)), block(bs);
        const T* tc = target + s0;
        T* qc = q + s0;
        int32_t* ic = iters ? iters + s0 : iters;
        T* ec = err ? err + s0 : err;
        if (at.trace) ar.trace = at.trace + s0;
        const int vr = a.with_rot == 2 ? 2 : a.with_rot ? 1 : 0, vg = GG == 1 ? 0 : GG == 2 ? 1 : GG == 4 ? 2 : 3;
        // (no_f64: the phase-2 kernel without the fp64 solve, where the launch never takes it -- see below)
        const hipFunction_t jk = !jf ? nullptr : no_f64 && jf->ik2[vr][vg] ? jf->ik2[vr][vg] : jf->ik[vr][vg];
        if (jk) {
            int64_t cc = c, pw = per_wave;
            void* args[] = {(void*)&ar, (void*)&tc, (void*)&ldt, (void*)&qc, (void*)&ldq, (void*)&cc,
                            (void*)&ic, (void*)&ec, (void*)&lde, (void*)&pw};
            return hipModuleLaunchKernel(jk, grid.x, 1, 1, (unsigned)bs, 1, 1, 0, st, args, nullptr);
        }
#define KIN_IK_G(MA, R, GX) \
        hipLaunchKernelGGL((k_ik_dls<T, MA, R, GX>), grid, block, 0, st, P, steps, ar, tc, ldt, qc, ldq, c, ic, ec, lde, per_wave)
#define KIN_IK6(MA) \
        switch (GG) { case 2: KIN_IK_G(MA, 6, 2); break; case 4: KIN_IK_G(MA, 6, 4); break; \
                      case 8: KIN_IK_G(MA, 6, 8); break; default: KIN_IK_G(MA, 6, 1); }
#define KIN_IK3(MA) \
        switch (GG) { case 2: KIN_IK_G(MA, 3, 2); break; case 4: KIN_IK_G(MA, 3, 4); break; \
                      case 8: KIN_IK_G(MA, 3, 8); break; default: KIN_IK_G(MA, 3, 1); }
        if (a.with_rot) {
            KIN_MAXA_DISPATCH(g.maxA, KIN_IK6)
        } else {
            KIN_MAXA_DISPATCH(g.maxA, KIN_IK3)
        }
#undef KIN_IK6
#undef KIN_IK3
#undef KIN_IK_G
        return hipGetLastError();
    };
    // lane byte offsets i * sizeof(T) stay below 2^32; with a scratch set, chunks of at most its capacity
    const int64_t chunk = scr.fail_list ? ik_chunk(a, scr.cap) : kIkChunk;
    for (int64_t s0 = 0; s0 < n; s0 += chunk) {
        at.ibase = a.index_base + s0;
        at.q0 = q0 ? q0 + s0 : nullptr;
        const int64_t c = std::min(chunk, n - s0);
        const int64_t ng = 64 / G;
        const int64_t plain = (c + ng - 1) / ng;
        // (automatic: batches that need more than one round of resident waves at G lanes per target
        // and fit the scratch list; phase 2 runs the remaining attempts side by side)
        const bool two = scr.fail_list && ik_two_phase(a, n, c, scr.cap);
        if (two) {
            // the ring's control words carry over from the previous call (no reset launch)
            hipError_t e;
            IkArgsT<T> a1 = at;  // phase 1: attempt 0, one lane per target
            a1.n_attempts = 1;
            a1.phase1 = 1;
            a1.fail_list = scr.fail_list;
            a1.fail_ctl = scr.fail_ctl;
            a1.fail_mask = (uint32_t)(scr.ring_cap - 1);
            a1.fail_aux = scr.fail_aux;
            // early hand-over (IkArgsT::p1_cut): attempt 0 stops after `cut` iterations in phase 1 and
            // phase 2 resumes it on slot 0 beside the other attempts.  Phase 1 then lasts `cut`
            // iterations instead of L and phase 2 (16 targets per wave at G = 4) absorbs the handed-over
            // ones at no extra latency while it stays within ~2 waves per SIMD (one wave alone issues
            // every other VALU slot).  Only while phase 1 is one round of resident waves: a larger
            // batch is throughput-bound, and the hand-over would add the speculative attempts 1, 2, ...
            // of every handed-over target that attempt 0 still solves (1M targets: 0.55 -> 0.59 ms).
            // Not for in-place calls of based plans (the hand-over would overwrite the start pose that
            // attempts 1, 2, ... begin from).
            const int cut = (c + 63) / 64 <= resident_waves ? ik_p1_cut(L, P.flags & PF_BASE ? (q0 != nullptr) : true, a.damp_err != 0.0) : 0;
            a1.p1_cut = cut;
            // phase 1 shares out targets like the one-phase schedule (one per lane while the batch
            // fills the chip in at most two rounds of waves, else wave-local queues) -- but a queue
            // of `resident_waves` waves must not run fewer waves per CU than the kernel could hold:
            // where the hardware keeps more resident (the fp32 specialised kernel, 3 per SIMD), the
            // full grid backfilled by the dispatcher is faster (profiles/r02_ik_queue_ab.txt)
            const int64_t plain1 = (c + 63) / 64;
            bool q1 = tpq_env != 0 && (qmode >= 0 ? qmode != 0 : plain1 > 2 * resident_waves);
            // The fp32 kernels solve attempt 0's first KINHIP_IK_F64_ITERS iterations in fp64: on a queue a
            // lane group that takes its next target runs those iterations while the rest of the wave is in
            // fp32, so nearly every wave iteration pays both solves.  The plain grid starts a wave's targets
            // together (1M targets: 0.607 -> 0.502 ms, identical results; profiles/r05_ik_1m_queue_ab.txt)
            if (sizeof(T) == 4 && KINHIP_IK_F64SOLVE == 3 && KINHIP_IK_F64_ITERS > 0 && tpq_env < 0 && qmode < 0)
                q1 = false;
            if (q1 && tpq_env < 0 && qmode < 0 && jf) {
                const hipFunction_t f1 = jf->ik[a.with_rot == 2 ? 2 : a.with_rot ? 1 : 0][0];
                int nb = 0;
                if (f1 && hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f1, 256, 0) == hipSuccess &&
                    (int64_t)nb * 4 * cus > resident_waves)
                    q1 = false;
            }
            const int64_t w1 = q1 ? std::min(resident_waves, plain1) : plain1;
            const int64_t pw1 = (c + w1 - 1) / w1;
            if ((e = one(a1, 1, s0, c, pw1, (c + pw1 - 1) / pw1)) != hipSuccess) return e;
            IkArgsT<T> a2 = at;  // phase 2: attempts 1.. (0 resumed, after a hand-over) of the listed targets
            a2.att0 = cut ? 0 : 1;
            a2.cont = cut ? 1 : 0;
            a2.p1_cut = cut;
            a2.fail_aux = scr.fail_aux;
            a2.idx = scr.fail_list;
            const int na2 = natt - a2.att0;
            const int G2 = na2 <= 1 ? 1 : na2 <= 2 ? 2 : na2 <= 4 ? 4 : 8;
            const int64_t ng2 = 64 / G2;
            // Phase 2's list fills only the first waves of its grid (one wave per SIMD or less).  Its waves
            // are dealt slot-major over the workgroups the chip holds at once (IkArgsT::p2_spread = the
            // phase-2 kernel's resident workgroups): the first wave of each, then the second, ... -- a
            // short list spreads over every CU, and a list of fewer waves than the resident workgroups
            // hold never reaches a workgroup that has to wait for a slot.  Round 4 dealt the list over the
            // WHOLE grid (4,096 workgroups at config 4): the fp64 kernel, two resident workgroups per CU,
            // then ran a 1,000-wave list in two rounds of one busy wave per workgroup (config 4 fp64
            // 0.145 -> 0.365 ms, BENCH_r04; A/B profiles/r05_ik_p2_ab.txt).  Measured (round 5,
            // profiles/r05_ik_p2_ab2.txt): the spread over the resident workgroups costs the fp32 kernels
            // (config 4 fixed lambda 0.071 -> 0.089 ms, damped 0.072 -> 0.084) and fp64 at fixed lambda (0.154
            // -> 0.163), and helps only damped fp64 (0.171 -> 0.158): every kernel runs block-major (round 3's
            // order).  KINHIP_IK_P2_SPREAD=<0 never (default) | 1 kernels of <= 2 resident workgroups per CU |
            // 2 always | 3 whole grid (round 4)>, KINHIP_IK_P2_BLOCK=<64|256> (A/B build).
            static const int p2_block_env = ab_env_int("KINHIP_IK_P2_BLOCK", 256);
            static const int spread_env = ab_env_int("KINHIP_IK_P2_SPREAD", 0);
            const int bs2 = p2_block_env == 64 ? 64 : 256;
            a2.p2_spread = 0;
            if (spread_env != 0 && bs2 == 256 && jf) {  // (the resident workgroups of the phase-2 kernel)
                const hipFunction_t f2 = jf->ik[a.with_rot == 2 ? 2 : a.with_rot ? 1 : 0][G2 == 1 ? 0 : G2 == 2 ? 1 : G2 == 4 ? 2 : 3];
                int nb = 0;
                if (f2 && hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f2, 256, 0) == hipSuccess && nb > 0 &&
                    (nb <= 2 || spread_env > 1))
                    a2.p2_spread = spread_env == 3 ? (int)(((c + ng2 - 1) / ng2 * 64 + 255) / 256)  // (A/B: whole grid)
                                                   : nb * cus;
            }
            a2.fail_ctl = scr.fail_ctl;
            a2.fail_mask = (uint32_t)(scr.ring_cap - 1);
            // Phase 2 never takes the fp32 kernels' fp64 solve (ik_body: attempt 0 before iteration
            // KINHIP_IK_F64_ITERS, or lambda^2 below KINHIP_IK_F32SOLVE_MIN_LAM2) when attempt 0 resumes at or past
            // that iteration and lambda is not below the threshold: its specialised form without that code
            // (F64S = false; the same arithmetic) then runs -- config 4 0.072-0.074 -> 0.070 ms on one box,
            // identical results (profiles/r06_ik_p2_nof64_ab.txt)
            const bool no_f64 = sizeof(T) == 4 && KINHIP_IK_F64SOLVE == 3 &&
                                !(at.lam2 < T(KINHIP_IK_F32SOLVE_MIN_LAM2)) && (cut == 0 || cut >= KINHIP_IK_F64_ITERS);
            if ((e = one(a2, G2, s0, c, ng2, (c + ng2 - 1) / ng2, bs2, no_f64)) != hipSuccess) {
                // phase 1 ran but phase 2 did not move the next call's start mark: restart the ring;
                // the targets phase 1 did not solve keep undefined outputs (kin_ik_dls_batch says so)
                (void)hipMemsetAsync(scr.fail_ctl, 0, sizeof(uint32_t) * kIkCtlStride * kIkSubRings, st);
                g_ik_partial = true;
                return e;
            }
            continue;
        }
        const bool queue = qmode >= 0 ? qmode != 0 : plain > 2 * resident_waves;
        const int64_t waves = queue ? std::min(resident_waves, plain) : plain;
        const int64_t per_wave = (c + waves - 1) / waves;  // targets each wave works through
        const int64_t nw = (c + per_wave - 1) / per_wave;
        const hipError_t e = one(at, G, s0, c, per_wave, nw);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <typename T>
hipError_t launch_nakamura(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const T* pts,
                           int64_t ldpt, T* q, int64_t ldq, int64_t n, const JitFns* jf, hipStream_t st) {
    for (int64_t s0 = 0; s0 < n; s0 += kChunk) {
        const int64_t c = std::min(kChunk, n - s0);
        const dim3 grid(grid_of(c, 256)), block(256);
        const T* pc = pts + s0;
        T* qc = q + s0;
        if (jf && jf->nakamura) {
            int64_t cc = c;
            void* args[] = {(void*)&pc, (void*)&ldpt, (void*)&qc, (void*)&ldq, (void*)&cc};
            const hipError_t e = hipModuleLaunchKernel(jf->nakamura, grid.x, 1, 1, 256, 1, 1, 0, st, args, nullptr);
            if (e != hipSuccess) return e;
            continue;
        }
#define KIN_NK_LAUNCH(MA) hipLaunchKernelGGL((k_nakamura<T, MA>), grid, block, 0, st, P, steps, pc, ldpt, qc, ldq, c)
        KIN_MAXA_DISPATCH(g.maxA, KIN_NK_LAUNCH)
#undef KIN_NK_LAUNCH
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

#define KIN_INSTANTIATE(T)                                                                                    \
    template hipError_t launch_ik_dls<T>(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const IkArgs&, \
                                         const T*, int64_t, const T*, T*, int64_t, int64_t, int32_t*, T*, int64_t, \
                                         const JitFns*, const IkScratch&, hipStream_t);                                         \
    template hipError_t launch_nakamura<T>(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const T*,    \
                                           int64_t, T*, int64_t, int64_t, const JitFns*, hipStream_t);
KIN_INSTANTIATE(float)
KIN_INSTANTIATE(double)

}  // namespace kinhip
