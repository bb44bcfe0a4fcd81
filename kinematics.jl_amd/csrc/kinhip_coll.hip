// kinhip_coll.hip -- k_coll: swept spheres vs a union of box SDFs, fused with FK.
// (gfx950 only; shared helpers in kinhip_device.h)
#include "kinhip_coll_dev.h"

namespace kinhip {
namespace {

// --------------------------------------------------------------------------
// generic kernel (the staged program is read from device memory)
// --------------------------------------------------------------------------
template <typename T, int MAXA, bool GRAD>
__global__ __launch_bounds__(256) void k_coll(const KProg<T> P, const KStep<T>* __restrict__ S,
                                              const KSphere<T>* __restrict__ sph, const KBox<T>* __restrict__ boxes,
                                              const CollArgs a, const T* __restrict__ q, int64_t ldq, int64_t n,
                                              T* __restrict__ dists, int64_t ldd, T* __restrict__ grads,
                                              int64_t ldg, T* __restrict__ min_dist, const Tiling tl) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    coll_body<T, MAXA, GRAD>(P, S, sph, boxes, a, q, ldq, n, dists, ldd, grads, ldg, min_dist, tl, smem);
}

// the same with the union's boxes attached to a scene mechanism (kin_coll_batch_scene; the plan-specialised
// form is kinhip_jit_colls_*, kinhip_jit.cpp)
template <typename T, int MAXA, bool GRAD>
__global__ __launch_bounds__(256) void k_coll_scene(const KProg<T> P, const KStep<T>* __restrict__ S,
                                                    const KSphere<T>* __restrict__ sph, const KBox<T>* __restrict__ boxes,
                                                    const CollArgs a, const T* __restrict__ q, int64_t ldq, int64_t n,
                                                    T* __restrict__ dists, int64_t ldd, T* __restrict__ grads,
                                                    int64_t ldg, T* __restrict__ min_dist, const Tiling tl,
                                                    const SceneArgs<T> sa) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    coll_body<T, MAXA, GRAD, kMaxSceneGroups>(P, S, sph, boxes, a, q, ldq, n, dists, ldd, grads, ldg, min_dist, tl, smem, sa);
}

}  // namespace

// KINHIP_COLL_LDS=<bytes> (A/B): reserve at least this much LDS per workgroup of the specialised
// collision kernels (an occupancy cap, as launch_fk's)
inline size_t coll_lds(size_t lds) {
    static const int env = [] {
        const int v = ab_env_int("KINHIP_COLL_LDS", -1);
        return v >= 0 && v <= 65536 ? v : -1;
    }();
    return env >= 0 && (size_t)env > lds ? (size_t)env : lds;
}

template <typename T>
hipError_t launch_coll_scene(const KProg<T>& P, const KStep<T>* steps, const KSphere<T>* sph, const KBox<T>* boxes,
                             const LaunchGeom& g, const CollArgs& a, const SceneLaunch& sl, const T* q, int64_t ldq,
                             int64_t n, T* dists, int64_t ldd, T* grads, int64_t ldg, T* min_dist, const JitFns* jf,
                             const JitFns* jfs, hipStream_t st) {
    const Tiling tl{0xffffffffu, 0, 0, 0, 0};
    const size_t lds = grads && a.n_boxes <= kCollLdsBoxes ? (size_t)a.n_boxes * sizeof(KBox<T>) : 0;
    for (int64_t s0 = 0; s0 < n; s0 += kChunk) {
        const int64_t c = std::min(kChunk, n - s0);
        const dim3 grid(grid_of(c, 256)), block(256);
        SceneArgs<T> sa;
        sa.groups = (const KSceneGroup*)sl.groups;
        sa.steps = (const KSceneStep<T>*)sl.steps;
        sa.q = (const T*)sl.q + (sl.uniform ? 0 : s0);
        sa.ld = sl.uniform ? 1 : sl.ld;  // uniform: the scene values are one column of cols entries
        sa.ng = sl.ng;
        sa.base_col = sl.base_col;
        sa.uniform = sl.uniform;
        const T* qc = q + s0;
        T* dc = dists ? dists + s0 : dists;
        T* gc = grads ? grads + s0 : grads;
        T* mc = min_dist ? min_dist + s0 : min_dist;
        // plan-specialised (kin_plan_specialize, KIN_SPEC_COLL): the 2-group kernel when the scene has at
        // most 2 moving groups (24 fewer registers for the per-lane group frames than the 4-group one)
        // kin_plan_specialize_scene (jfs): this union's tables compiled in as well
        const hipFunction_t jsc = jfs ? jfs->coll_scene_c[grads ? 1 : 0] : nullptr;
        const hipFunction_t jk = jsc ? jsc : jf ? jf->coll_scene[grads ? 1 : 0][sl.ng <= 2 ? 0 : 1] : nullptr;
        if (jk) {
            // the 2-group kernel keeps its lanes' group frames in LDS after the boxes (coll_body, SceneCtx)
            static const bool frames_lds = ab_env_int("KINHIP_SCENE_LDS", 0) != 0;  // (A/B build; see kinhip_jit.cpp)
            const size_t ldsj = sl.ng <= 2 && frames_lds && scene_frames_in_lds<T>(2)
                                    ? (lds + 15) / 16 * 16 + 2 * 12 * 256 * sizeof(T)
                                    : lds;
            int64_t cc = c;
            CollArgs ac = a;
            Tiling tc = tl;
            void* args[] = {(void*)&boxes, (void*)&ac, (void*)&qc, (void*)&ldq, (void*)&cc, (void*)&dc, (void*)&ldd,
                            (void*)&gc, (void*)&ldg, (void*)&mc, (void*)&tc, (void*)&sa};
            const hipError_t e = hipModuleLaunchKernel(jk, grid.x, 1, 1, 256, 1, 1,
                                                       (unsigned)coll_lds(ldsj), st, args, nullptr);
            if (e != hipSuccess) return e;
            continue;
        }
#define KIN_COS_LAUNCH(MA) \
        hipLaunchKernelGGL((k_coll_scene<T, MA, false>), grid, block, lds, st, P, steps, sph, boxes, a, qc, ldq, c, dc, ldd, gc, ldg, mc, tl, sa)
#define KIN_COSG_LAUNCH(MA) \
        hipLaunchKernelGGL((k_coll_scene<T, MA, true>), grid, block, lds, st, P, steps, sph, boxes, a, qc, ldq, c, dc, ldd, gc, ldg, mc, tl, sa)
        if (grads) {
            KIN_MAXA_DISPATCH(g.maxA, KIN_COSG_LAUNCH)
        } else {
            KIN_MAXA_DISPATCH(g.maxA, KIN_COS_LAUNCH)
        }
#undef KIN_COS_LAUNCH
#undef KIN_COSG_LAUNCH
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <typename T>
hipError_t launch_coll(const KProg<T>& P, const KStep<T>* steps, const KSphere<T>* sph, const KBox<T>* boxes,
                       const LaunchGeom& g, const CollArgs& a, const T* q, int64_t ldq, int64_t n, T* dists,
                       int64_t ldd, T* grads, int64_t ldg, T* min_dist, const TileArgs& ta, const JitFns* jf,
                       hipStream_t st) {
    // plain SoA (tile >= n): chunks are element offsets along the rows; tiled: whole tiles per chunk
    const bool tiled = ta.tile < n;
    const int64_t chunk = tiled ? (kChunk / ta.tile) * ta.tile : kChunk;
    Tiling tl{tiled ? (uint32_t)(ta.tile / 256) : 0xffffffffu, ta.tsq, ta.tsp, ta.tsj, ta.tsm};
    // distances + gradients: the union's boxes in LDS (coll_body, kCollLdsBoxes)
    const size_t lds = grads && a.n_boxes <= kCollLdsBoxes ? (size_t)a.n_boxes * sizeof(KBox<T>) : 0;
    for (int64_t s0 = 0; s0 < n; s0 += chunk) {
        const int64_t c = std::min(chunk, n - s0);
        const dim3 grid(grid_of(c, 256)), block(256);
        const int64_t nt = tiled ? s0 / ta.tile : 0;
        const T* qc = q + (tiled ? nt * ta.tsq : s0);
        T* dc = dists ? dists + (tiled ? nt * ta.tsp : s0) : dists;
        T* gc = grads ? grads + (tiled ? nt * ta.tsj : s0) : grads;
        T* mc = min_dist ? min_dist + (tiled ? nt * ta.tsm : s0) : min_dist;
        if (jf && jf->coll[grads ? 1 : 0]) {
            int64_t cc = c;
            CollArgs ac = a;
            void* args[] = {(void*)&boxes, (void*)&ac, (void*)&qc, (void*)&ldq, (void*)&cc, (void*)&dc,
                            (void*)&ldd, (void*)&gc, (void*)&ldg, (void*)&mc, (void*)&tl};
            const hipError_t e =
                hipModuleLaunchKernel(jf->coll[grads ? 1 : 0], grid.x, 1, 1, 256, 1, 1, (unsigned)coll_lds(lds), st,
                                      args, nullptr);
            if (e != hipSuccess) return e;
            continue;
        }
#define KIN_CO_LAUNCH(MA) \
        hipLaunchKernelGGL((k_coll<T, MA, false>), grid, block, lds, st, P, steps, sph, boxes, a, qc, ldq, c, dc, ldd, gc, ldg, mc, tl)
#define KIN_COG_LAUNCH(MA) \
        hipLaunchKernelGGL((k_coll<T, MA, true>), grid, block, lds, st, P, steps, sph, boxes, a, qc, ldq, c, dc, ldd, gc, ldg, mc, tl)
        if (grads) {
            KIN_MAXA_DISPATCH(g.maxA, KIN_COG_LAUNCH)
        } else {
            KIN_MAXA_DISPATCH(g.maxA, KIN_CO_LAUNCH)
        }
#undef KIN_CO_LAUNCH
#undef KIN_COG_LAUNCH
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

#define KIN_INSTANTIATE(T)                                                                                    \
    template hipError_t launch_coll<T>(const KProg<T>&, const KStep<T>*, const KSphere<T>*, const KBox<T>*,   \
                                       const LaunchGeom&, const CollArgs&, const T*, int64_t, int64_t, T*,    \
                                       int64_t, T*, int64_t, T*, const TileArgs&, const JitFns*, hipStream_t); \
    template hipError_t launch_coll_scene<T>(const KProg<T>&, const KStep<T>*, const KSphere<T>*, const KBox<T>*, \
                                             const LaunchGeom&, const CollArgs&, const SceneLaunch&, const T*,        \
                                             int64_t, int64_t, T*, int64_t, T*, int64_t, T*, const JitFns*,     \
                                             const JitFns*, hipStream_t);
KIN_INSTANTIATE(float)
KIN_INSTANTIATE(double)

}  // namespace kinhip
