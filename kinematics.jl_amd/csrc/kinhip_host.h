// kinhip_host.h -- internal host helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "kinhip_prog.h"

namespace kinhip {
// Records a thread-local message for kin_last_error() and returns code.
int set_error(int code, const std::string& msg);

// plan specialisation (kinhip_jit.cpp): kernels compiled for one staged program
struct JitKernels;
struct JitFns;
template <typename T>
int jit_build(const KProg<T>& P, const KStep<T>* steps, int nsteps, int maxA, const void* spheres, int n_sph,
              const KIkcProg<T>* ikc, const void* ikc_steps, const void* ikc_sph, uint32_t kernels, JitKernels** out);
// the k_coll_scene kernels of one staged collision program with one attached union's tables (groups,
// scene steps, boxes, axis-aligned boxes) as constants: kin_plan_specialize_scene
struct JitScene {
    const KSceneGroup* groups;
    int ng;
    const void* steps;  // KSceneStep<T>[ns]
    int ns;
    const void* boxes;  // KBox<T>[nb]
    int nb;
    const void* aabb;   // KAabb<T>[na]
    int na;
    int base_col;
};
template <typename T>
int jit_build_scene(const KProg<T>& P, const KStep<T>* steps, int nsteps, int maxA, const void* spheres, int n_sph,
                    const JitScene& sc, JitKernels** out);
void jit_destroy(JitKernels* k);
const JitFns* jit_fns(const JitKernels* k);  // null for a null k
int jit_selfcheck();
}  // namespace kinhip
