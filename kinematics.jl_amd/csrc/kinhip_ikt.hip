// kinhip_ikt.hip -- k_ik_tree (batched collision-aware IK, stage 2 of the reference's bistage
// inverse_kinematics!, src/inverse_kinematics.jl:1-21): the generic kernels and the launcher of the
// generic and plan-specialised forms.  (gfx950 only; the body is kinhip_ikt_dev.h.)
#include "kinhip_ikt_dev.h"

namespace kinhip {
namespace {

// Generic collision-aware IK: the program from memory, one sphere lane per target and G attempt groups
// (G = 1: attempts in sequence; G = 4: a target's restart attempts side by side, kin_ik_params.lanes
// 2 / 4 / 8 -- identical results).  MAXV bounds the variables (normal equations in registers: 8, 12 or
// kIkcMaxVars); MAXG > 0: boxes attached to a scene, scene joint values per target.
template <typename T, int MAXV, int ROWS, int G, int MAXG>
__global__ __launch_bounds__(64) void k_ik_tree(const KIkcProg<T> P, const KIkcStep<T>* __restrict__ S,
                                                const KSphere<T>* __restrict__ sph, const KBox<T>* __restrict__ boxes,
                                                const CollArgs ca, const IkcArgsT<T> cz, const IkArgsT<T> a,
                                                const SceneArgs<T> sa, const T* __restrict__ tgt, int64_t ldt,
                                                T* __restrict__ q, int64_t ldq, int64_t n, int32_t* __restrict__ iters,
                                                T* __restrict__ err, int64_t lde) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    ikt_body<T, MAXV, ROWS, G, 1, 1, MAXG>(P, S, sph, boxes, ca, cz, a, sa, tgt, ldt, q, ldq, n, iters, err, lde, smem);
}

}  // namespace

// Lanes of a k_ik_tree target (specialised kernels): G attempt groups run a target's restart attempts
// side by side, S sphere lanes per group share out its spheres -- identical results for every (S, G).
// Small batches fill the chip only this way (the bistage solve's few thousand targets are a fraction of
// a wave per SIMD): G = 4 while there are restart attempts and up to 2^16 targets, S = 16 while the
// whole batch stays within ~4 waves per SIMD (n * G * 16 <= 2^18 lanes), else S = 1.
// kin_ik_params.lanes forces a form: 1 = one lane, 2 / 4 / 8 = 4 attempt groups of one lane, 16 = 16
// sphere lanes x 1, 64 = 16 x 4; KINHIP_IKT_S / KINHIP_IKT_G override (A/B build).
static int ikt_variant(int64_t n, int natt, int lanes) {
    static const int s_env = ab_env_int("KINHIP_IKT_S", 0), g_env = ab_env_int("KINHIP_IKT_G", 0);
    if (lanes == 1) return 0;
    if (lanes == 2 || lanes == 4 || lanes == 8) return 1;
    if (lanes == 16) return 2;
    if (lanes == 64) return 3;
    int G = natt >= 2 && n <= (int64_t(1) << 16) ? 4 : 1;
    int S = n * G * 16 <= (int64_t(1) << 18) ? 16 : 1;
    if (s_env) S = s_env;
    if (g_env) G = g_env;
    for (int v = 0; v < kIktVariants; ++v)
        if (kIktS[v] == S && kIktG[v] == G) return v;
    return 0;
}

template <typename T>
hipError_t launch_ik_tree(const KIkcProg<T>& P, const KIkcStep<T>* steps, const KSphere<T>* sph, const KBox<T>* boxes,
                          const CollArgs& ca, const SceneLaunch* scene, const IkcArgs& c, const IkArgs& a,
                          const T* target, int64_t ldt, const T* q0, T* q, int64_t ldq, int64_t n, int32_t* iters,
                          T* err, int64_t lde, const JitFns* jf, hipStream_t st) {
    int L, natt;
    ik_attempts(a, &L, &natt);
    IkArgsT<T> at{a.max_iters, T(a.lambda * a.lambda), T(a.tol_pos), T(a.tol_rot), T(a.max_step), L, natt, a.seed,
                  0, 0, 0, nullptr, nullptr, nullptr, 0u, nullptr, a.with_rot == 2 ? 1 : 0};
    const IkcArgsT<T> cz{T(c.margin), T(c.band), T(c.weight), T(c.feas)};
    const size_t lds = ca.n_boxes <= kCollLdsBoxes ? (size_t)ca.n_boxes * sizeof(KBox<T>) : 0;
    const int rows6 = a.with_rot ? 1 : 0;
    // specialised kernels: the static union (ikt), a union attached to a scene of at most 2 moving groups
    // (ikts, KIN_SPEC_IK_COLL_SCENE); a scene of more groups runs the generic kernel
    const int vi = jf ? ikt_variant(n, natt, a.lanes) : 0;
    const hipFunction_t jk = !jf ? nullptr : !scene ? jf->ikt[rows6][vi] : scene->ng <= 2 ? jf->ikts[rows6][vi] : nullptr;
    // generic kernel: attempt groups side by side only when the caller asks for them (lanes 2 / 4 / 8)
    const int gg = (a.lanes == 2 || a.lanes == 4 || a.lanes == 8) && natt > 1 && P.nv <= 12 ? 4 : 1;
    const int lanes = jk ? kIktS[vi] * kIktG[vi] : gg;
    SceneArgs<T> sa{};
    if (scene) {
        sa.groups = (const KSceneGroup*)scene->groups;
        sa.steps = (const KSceneStep<T>*)scene->steps;
        sa.q = (const T*)scene->q;
        sa.ld = scene->ld;
        sa.ng = scene->ng;
        sa.base_col = scene->base_col;
        sa.uniform = scene->uniform;
    }
    for (int64_t s0 = 0; s0 < n; s0 += kIkChunk) {
        const int64_t cn = std::min(kIkChunk, n - s0);
        at.ibase = a.index_base + s0;
        at.q0 = q0 ? q0 + s0 : nullptr;
        at.q_alt = a.q_alt ? (const T*)a.q_alt + s0 : nullptr;
        const T* tc = target + s0;
        T* qc = q + s0;
        int32_t* ic = iters ? iters + s0 : iters;
        T* ec = err ? err + s0 : err;
        SceneArgs<T> sac = sa;
        if (scene && !sa.uniform) sac.q = sa.q + s0;
        const unsigned grid = (unsigned)((cn * lanes + 63) / 64);
        if (jk) {
            int64_t cc = cn;
            CollArgs cac = ca;
            IkcArgsT<T> czc = cz;
            void* args_static[] = {(void*)&boxes, (void*)&cac, (void*)&czc, (void*)&at, (void*)&tc, (void*)&ldt,
                                   (void*)&qc, (void*)&ldq, (void*)&cc, (void*)&ic, (void*)&ec, (void*)&lde};
            void* args_scene[] = {(void*)&boxes, (void*)&cac, (void*)&czc, (void*)&at, (void*)&tc, (void*)&ldt,
                                  (void*)&qc, (void*)&ldq, (void*)&cc, (void*)&ic, (void*)&ec, (void*)&lde, (void*)&sac};
            const hipError_t e = hipModuleLaunchKernel(jk, grid, 1, 1, 64, 1, 1, (unsigned)lds, st,
                                                       scene ? args_scene : args_static, nullptr);
            if (e != hipSuccess) return e;
            continue;
        }
#define KIN_IKT(MV, R, GG, MG) \
        hipLaunchKernelGGL((k_ik_tree<T, MV, R, GG, MG>), dim3(grid), dim3(64), lds, st, P, steps, sph, boxes, ca, cz, at, sac, tc, ldt, qc, ldq, cn, ic, ec, lde)
#define KIN_IKT_G(MV, MG)                                                          \
        if (a.with_rot) {                                                          \
            if (gg == 4) KIN_IKT(MV, 6, 4, MG); else KIN_IKT(MV, 6, 1, MG);        \
        } else {                                                                   \
            if (gg == 4) KIN_IKT(MV, 3, 4, MG); else KIN_IKT(MV, 3, 1, MG);        \
        }
#define KIN_IKT_1(MV, MG)                                  \
        if (a.with_rot) KIN_IKT(MV, 6, 1, MG); else KIN_IKT(MV, 3, 1, MG);
        // (variables bound 8, 12 or kIkcMaxVars: the normal equations and joint records live in registers,
        // spilled to scratch beyond 12 in the generic kernels -- the parity path of wide trees; their
        // specialised forms fold the structural zeros of the system.  Wide trees run one lane group.)
        if (scene) {
            if (P.nv <= 12) { KIN_IKT_G(12, kMaxSceneGroups) } else { KIN_IKT_1(kIkcMaxVars, kMaxSceneGroups) }
        } else if (P.nv <= 8) {
            KIN_IKT_G(8, 0)
        } else if (P.nv <= 12) {
            KIN_IKT_G(12, 0)
        } else {
            KIN_IKT_1(kIkcMaxVars, 0)
        }
#undef KIN_IKT_1
#undef KIN_IKT_G
#undef KIN_IKT
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

#define KIN_INSTANTIATE(T)                                                                                  \
    template hipError_t launch_ik_tree<T>(const KIkcProg<T>&, const KIkcStep<T>*, const KSphere<T>*,        \
                                          const KBox<T>*, const CollArgs&, const SceneLaunch*, const IkcArgs&, \
                                          const IkArgs&, const T*, int64_t, const T*, T*, int64_t, int64_t,    \
                                          int32_t*, T*, int64_t, const JitFns*, hipStream_t);
KIN_INSTANTIATE(float)
KIN_INSTANTIATE(double)

}  // namespace kinhip
