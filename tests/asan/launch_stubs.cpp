// Test-only: the host sanitizer harness links the engine's host translation units (kinhip_host.cpp,
// kinhip_urdf.cpp, kinhip_jit.cpp) without the gfx950 kernel TUs; these launchers stand in for them and
// report "no device" (a plan never reaches them in a sanitizer run: staging needs a device first).
#include "kinhip_internal.h"

namespace kinhip {
template <typename T>
hipError_t launch_fk(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const T*, int64_t, int64_t, T*, int64_t,
                     T*, int64_t, const TileArgs&, const JitFns*, hipStream_t) {
    return hipErrorNoDevice;
}
template <typename T>
hipError_t launch_ik_dls(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const IkArgs&, const T*, int64_t,
                         const T*, T*, int64_t, int64_t, int32_t*, T*, int64_t, const JitFns*, const IkScratch&,
                         hipStream_t) {
    return hipErrorNoDevice;
}
template <typename T>
hipError_t launch_ik_tree(const KIkcProg<T>&, const KIkcStep<T>*, const KSphere<T>*, const KBox<T>*, const CollArgs&,
                          const SceneLaunch*, const IkcArgs&, const IkArgs&, const T*, int64_t, const T*, T*, int64_t,
                          int64_t, int32_t*, T*, int64_t, const JitFns*, hipStream_t) {
    return hipErrorNoDevice;
}
bool ik_wants_two_phase(const IkArgs&, int64_t, int64_t) { return false; }
bool ik_last_call_partial() { return false; }
template <typename T>
hipError_t launch_nakamura(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const T*, int64_t, T*, int64_t,
                           int64_t, const JitFns*, hipStream_t) {
    return hipErrorNoDevice;
}
template <typename T>
hipError_t launch_coll(const KProg<T>&, const KStep<T>*, const KSphere<T>*, const KBox<T>*, const LaunchGeom&,
                       const CollArgs&, const T*, int64_t, int64_t, T*, int64_t, T*, int64_t, T*, const TileArgs&,
                       const JitFns*, hipStream_t) {
    return hipErrorNoDevice;
}
template <typename T>
hipError_t launch_coll_scene(const KProg<T>&, const KStep<T>*, const KSphere<T>*, const KBox<T>*, const LaunchGeom&,
                             const CollArgs&, const SceneLaunch&, const T*, int64_t, int64_t, T*, int64_t, T*, int64_t,
                             T*, const JitFns*, const JitFns*, hipStream_t) {
    return hipErrorNoDevice;
}
template <typename T>
hipError_t launch_pose_residual(const T*, int64_t, const T*, int64_t, int64_t, int, T*, int64_t, hipStream_t) {
    return hipErrorNoDevice;
}
#define KIN_STUBS(T)                                                                                                 \
    template hipError_t launch_fk<T>(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const T*, int64_t,        \
                                     int64_t, T*, int64_t, T*, int64_t, const TileArgs&, const JitFns*, hipStream_t); \
    template hipError_t launch_ik_dls<T>(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const IkArgs&,        \
                                         const T*, int64_t, const T*, T*, int64_t, int64_t, int32_t*, T*, int64_t,  \
                                         const JitFns*, const IkScratch&, hipStream_t);                              \
    template hipError_t launch_ik_tree<T>(const KIkcProg<T>&, const KIkcStep<T>*, const KSphere<T>*, const KBox<T>*, \
                                          const CollArgs&, const SceneLaunch*, const IkcArgs&, const IkArgs&,        \
                                          const T*, int64_t, const T*, T*, int64_t, int64_t, int32_t*, T*, int64_t,   \
                                          const JitFns*, hipStream_t);                                               \
    template hipError_t launch_nakamura<T>(const KProg<T>&, const KStep<T>*, const LaunchGeom&, const T*, int64_t, \
                                           T*, int64_t, int64_t, const JitFns*, hipStream_t);                       \
    template hipError_t launch_coll<T>(const KProg<T>&, const KStep<T>*, const KSphere<T>*, const KBox<T>*,         \
                                       const LaunchGeom&, const CollArgs&, const T*, int64_t, int64_t, T*, int64_t, \
                                       T*, int64_t, T*, const TileArgs&, const JitFns*, hipStream_t);               \
    template hipError_t launch_coll_scene<T>(const KProg<T>&, const KStep<T>*, const KSphere<T>*, const KBox<T>*,   \
                                             const LaunchGeom&, const CollArgs&, const SceneLaunch&, const T*,        \
                                             int64_t, int64_t, T*, int64_t, T*, int64_t, T*, const JitFns*,      \
                                             const JitFns*, hipStream_t);                                             \
    template hipError_t launch_pose_residual<T>(const T*, int64_t, const T*, int64_t, int64_t, int, T*, int64_t,    \
                                                hipStream_t);
KIN_STUBS(float)
KIN_STUBS(double)
}  // namespace kinhip
