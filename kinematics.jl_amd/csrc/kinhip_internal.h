// kinhip_internal.h -- host-side launch entry points of the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kinhip_prog.h"

namespace kinhip {

// A/B knobs (schedules, occupancy, trig / atan variants, extra compiler options) are read from the
// environment only by the tools build (`make ab` -> lib/libkinhip_ab.so, -DKINHIP_AB_KNOBS=1,
// driven by tools/ab.py).  The product library never reads them: a stray environment variable
// cannot change a drop-in library's schedule or arithmetic.
#ifndef KINHIP_AB_KNOBS
#define KINHIP_AB_KNOBS 0
#endif
inline const char* ab_env(const char* name) {
#if KINHIP_AB_KNOBS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}
inline int ab_env_int(const char* name, int dflt) {
    const char* e = ab_env(name);
    return e ? atoi(e) : dflt;
}

// phase-A chain bounds compiled into the kernels (kinhip_device.h KIN_MAXA_DISPATCH)
inline int pick_chain_bound(int n) { return n <= 4 ? 4 : n <= 8 ? 8 : n <= 12 ? 12 : n <= 16 ? 16 : 32; }

struct LaunchGeom {
    int block;      // threads per workgroup (multiple of 64)
    size_t lds;     // dynamic LDS bytes
    int maxA;       // phase-A steps as compiled (4 / 8 / 12 / 16 / 32); the program is padded to it
};

// Tiled SoA (kin_plan_run_tiled): element (i, r) of an array at (i / tile) * ts + r * ld + i % tile.
// tile >= n is the plain SoA of kin_plan_run (one tile, ts unused).
struct TileArgs {
    int64_t tile;
    int64_t tsq, tsp, tsj;  // tile strides (elements) of q, poses / dists, jac / grads
    int64_t tsm = 0;        // min_dist (k_coll)
};
inline TileArgs plain_soa(int64_t n) { return TileArgs{n, 0, 0, 0, 0}; }

// Plan-specialised kernels of one plan (kinhip_jit.cpp); a null entry means
// the generic kernel runs.
struct JitFns {
    hipFunction_t fk = nullptr;
    hipFunction_t fk_stride = nullptr;  // the same, grid-strided with prefetched angles (launch_fk)
    hipFunction_t ik[3][4] = {};  // [0: rows 3, 1: rows 6 axis-angle, 2: rows 6 rpy objective][log2 of lanes per target]
    hipFunction_t ik2[3][4] = {};  // the same without the fp64 solve (phase 2 of launch_ik_dls; G >= 2 only)
    hipFunction_t nakamura = nullptr;
    hipFunction_t coll[2] = {};   // [with gradients]
    hipFunction_t coll_scene[2][2] = {};  // the same over an attached union [with gradients][up to 2 | 4 groups]
    // the same with one attached union's tables compiled in (kin_plan_specialize_scene) [with gradients]
    hipFunction_t coll_scene_c[2] = {};
    // collision-aware IK (k_ik_tree) [rows == 6][lanes: 0 = 1 x 1, 1 = 1 sphere lane x 4 attempt groups,
    // 2 = 16 sphere lanes x 1, 3 = 16 x 4] (kIktVariants)
    hipFunction_t ikt[2][4] = {};
    hipFunction_t ikts[2][4] = {};  // the same over a union attached to a scene of at most 2 moving groups
};
// sphere lanes S and attempt groups G of the specialised k_ik_tree kernels, by JitFns::ikt index
constexpr int kIktVariants = 4;
constexpr int kIktS[kIktVariants] = {1, 1, 16, 16};
constexpr int kIktG[kIktVariants] = {1, 4, 1, 4};

// jf: the plan-specialised kernels (kinhip_jit.cpp) or null for the generic one
template <typename T>
hipError_t launch_fk(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const T* q, int64_t ldq,
                     int64_t n, T* poses, int64_t ldp, T* jac, int64_t ldj, const TileArgs& ta, const JitFns* jf,
                     hipStream_t st);

struct IkArgs {
    int32_t max_iters;
    double lambda, tol_pos, tol_rot, max_step;
    int32_t with_rot;
    int32_t restarts;
    uint64_t seed;
    int32_t lanes;  // 0 auto
    int64_t index_base;  // global index of target 0 (restart draws)
    double damp_err;     // error-scaled damping (k_ik_dls only)
    void* trace = nullptr;  // kin_ik_dls_batch_trace: [2 (max_iters + 1)][trace_ld] residual norms per iterate
    int64_t trace_ld = 0;
    const void* q_alt = nullptr;  // kin_ik_coll_batch_alt: attempt 1's start pose (same layout as q), or null
};

// restart schedule of kin_ik_params: attempt length L (0: no restarts) and the attempts it reaches
inline void ik_attempts(const IkArgs& a, int* L, int* natt) {
    *L = a.restarts > 0 ? a.max_iters / (a.restarts + 1) : 0;
    *natt = (*L > 0 && a.max_iters > 0) ? 1 + (a.max_iters - 1) / *L : 1;
}

// Device scratch of the two-phase IK schedule (launch_ik_dls): the list of targets attempt 0 did
// not solve and its length, for batches of up to `cap` targets (null: single phase only)
struct IkScratch {
    int32_t* fail_list = nullptr;  // kIkSubRings rings of ring_cap entries (IkArgsT)
    int32_t* fail_aux = nullptr;   // per ring entry: the handed-over active set (IkArgsT::p1_cut)
    uint32_t* fail_ctl = nullptr;  // per ring 3 control words on a 128-byte line, zero at allocation
    int64_t cap = 0;               // targets per call the rings can take (a chunk of at most cap runs two-phase)
    int64_t ring_cap = 0;          // entries per ring, a power of two
};

// true when some chunk of an n-target kin_ik_dls_batch call runs the two-phase schedule (only then
// does the call need the plan's scratch ring)
bool ik_wants_two_phase(const IkArgs& a, int64_t n, int64_t cap);
// true when the last launch_ik_dls of this thread failed after its phase 1 had been launched (the
// targets phase 1 did not solve then keep undefined outputs)
bool ik_last_call_partial();

template <typename T>
hipError_t launch_ik_dls(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const IkArgs& a,
                         const T* target, int64_t ldt, const T* q0, T* q, int64_t ldq, int64_t n, int32_t* iters,
                         T* err, int64_t lde, const JitFns* jf, const IkScratch& scr, hipStream_t st);

// collision-aware IK (k_ik_tree, kinhip_ikt_dev.h): sphere-distance bound and penalty rows
struct IkcArgs {
    double margin, band, weight, feas;
};
struct SceneLaunch;

// scene: boxes attached to a scene mechanism, scene joint values per target (null: a static union)
template <typename T>
hipError_t launch_ik_tree(const KIkcProg<T>& P, const KIkcStep<T>* steps, const KSphere<T>* sph, const KBox<T>* boxes,
                          const CollArgs& ca, const SceneLaunch* scene, const IkcArgs& c, const IkArgs& a,
                          const T* target, int64_t ldt, const T* q0, T* q, int64_t ldq, int64_t n, int32_t* iters,
                          T* err, int64_t lde, const JitFns* jf, hipStream_t st);

template <typename T>
hipError_t launch_nakamura(const KProg<T>& P, const KStep<T>* steps, const LaunchGeom& g, const T* pts,
                           int64_t ldpt, T* q, int64_t ldq, int64_t n, const JitFns* jf, hipStream_t st);


template <typename T>
hipError_t launch_coll(const KProg<T>& P, const KStep<T>* steps, const KSphere<T>* sph, const KBox<T>* boxes,
                       const LaunchGeom& g, const CollArgs& a, const T* q, int64_t ldq, int64_t n, T* dists,
                       int64_t ldd, T* grads, int64_t ldg, T* min_dist, const TileArgs& ta, const JitFns* jf,
                       hipStream_t st);

// kin_coll_batch_scene: the scene side of k_coll_scene (device tables of the kin_sdf, scene columns)
struct SceneLaunch {
    const void* groups;  // KSceneGroup[ng]
    const void* steps;   // KSceneStep<T>[]
    const void* q;       // scene columns [cols][ld]
    int64_t ld;
    int32_t ng, base_col, uniform;
};
template <typename T>
hipError_t launch_coll_scene(const KProg<T>& P, const KStep<T>* steps, const KSphere<T>* sph, const KBox<T>* boxes,
                             const LaunchGeom& g, const CollArgs& a, const SceneLaunch& sl, const T* q, int64_t ldq,
                             int64_t n, T* dists, int64_t ldd, T* grads, int64_t ldg, T* min_dist, const JitFns* jf,
                             const JitFns* jfs, hipStream_t st);

template <typename T>
hipError_t launch_pose_residual(const T* poses, int64_t ldp, const T* target, int64_t ldt, int64_t n, int rows, T* vals,
                                int64_t ldv, hipStream_t st);

}  // namespace kinhip
