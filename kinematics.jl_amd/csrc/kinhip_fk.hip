// kinhip_fk.hip -- k_fk (batched get_transform + get_jacobian!) and k_pose_residual.
// (gfx950 only; shared helpers in kinhip_device.h)
#include "kinhip_fk_dev.h"

namespace kinhip {
namespace {

// --------------------------------------------------------------------------
// k_fk: generic kernel (the staged program is read from device memory)
// --------------------------------------------------------------------------
template <typename T, int MAXA>
__global__ __launch_bounds__(256) void k_fk(const KProg<T> P, const KStep<T>* __restrict__ S,
                                            const T* __restrict__ q, int64_t ldq, int64_t n,
                                            T* __restrict__ poses, int64_t ldp, T* __restrict__ jac,
                                            int64_t ldj, const Tiling tl) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    fk_body<T, MAXA>(P, S, reinterpret_cast<T*>(smem), q, ldq, n, poses, ldp, jac, ldj, tl);
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
                     int64_t n, T* poses, int64_t ldp, T* jac, int64_t ldj, const TileArgs& ta, const JitFns* jf,
                     hipStream_t st) {
    // Rounds 2-5 ran batches whose arrays far exceed the 256 MiB Infinity Cache (2^23 and up) on the
    // grid-strided specialised kernel with 2 configurations per lane, the next configuration's angles in
    // flight while this one is computed and stored (then 2^24 fp32 FK + J 799 -> 733 us; 2^20 41 vs 46 us for
    // the one-per-lane grid; tools/fk_stride_ab.py, profiles/r02_fk_stride_ab.txt).
    // Since the occupancy cap below (round 4) the one-per-lane grid is the faster one at every size, and only it
    // runs: fp32 2^24 670 vs 735 us, 2^26 2677 vs 2851 us; fp64 2^24 1321 vs 1763 us, 2^26 5270 vs 6817 us; 2^20 /
    // 2^22 equal (profiles/r06_fk_stride_ab.txt).  The grid-strided kernel stays for A/B runs:
    // KINHIP_FK_PER_LANE=<k> forces k configurations per lane (1: the plain kernel).
    static const int per_lane_env = [] {
        const int v = ab_env_int("KINHIP_FK_PER_LANE", 0);
        return v >= 1 && v <= 64 ? v : 0;
    }();
    // Occupancy: the specialised one-configuration-per-lane kernel reserves 64 KB of (unused) LDS per
    // 256-lane workgroup, so a CU holds 2 workgroups (8 waves, 2 per SIMD; 160 KB of LDS per CU): with fewer
    // lanes streaming 8 rows in and 60 out at once, HBM serves them faster -- 2^20 FK + J 41.5 -> 40.6 us,
    // 2^22 161 -> 153.5 us, fp64 6-link FK 107.5 -> 100.2 us; the grid-strided kernel (2^23+) keeps its
    // full occupancy (730 vs 746 us capped), as does the pattern probe's own sweep (bench.py PROBE_LDS,
    // profiles/r04_fk_occupancy_ab.txt, r04_ik_solve_probe_occ_ab.txt).
    // KINHIP_FK_LDS=<bytes> (A/B) overrides the reservation of both specialised kernels.
    constexpr unsigned kFkLds = 65536;
    static const int fk_lds_env = [] {
        const int v = ab_env_int("KINHIP_FK_LDS", -1);
        return v >= 0 && v <= 65536 ? v : -1;
    }();
    // fp64: 128-lane workgroups for the one-per-lane specialised kernel (with the 64 KB reservation: 4 waves
    // per CU, 1 per SIMD): config 2's fp64 FK of 6 links 101-104 -> 94 us; fp32 keeps 256 (44 us at 128)
    // (profiles/r04_fk_block_probe_ab.txt).  KINHIP_FK_BLOCK=<64|128|256> (A/B) overrides.
    static const int fk_block_env = [] {
        const int v = ab_env_int("KINHIP_FK_BLOCK", 0);
        return v == 64 || v == 128 || v == 256 ? v : 0;
    }();
    const bool one_per_lane = !(per_lane_env > 1);
    const int want = fk_block_env ? fk_block_env : (sizeof(T) == 8 && one_per_lane ? 128 : g.block);
    const int blk = jf && jf->fk && (ta.tile >= n || ta.tile % want == 0) ? want : g.block;  // (tiles: whole blocks)
    // plain SoA (tile >= n): chunks are element offsets along the rows; tiled: whole tiles per chunk
    const bool tiled = ta.tile < n;
    const int64_t chunk = tiled ? (kChunk / ta.tile) * ta.tile : kChunk;
    Tiling tl{tiled ? (uint32_t)(ta.tile / blk) : 0xffffffffu, ta.tsq, ta.tsp, ta.tsj, 0};
    for (int64_t s0 = 0; s0 < n; s0 += chunk) {
        const int64_t c = std::min(chunk, n - s0);
        const dim3 grid(grid_of(c, blk)), block(blk);
        const int64_t tq = tiled ? (s0 / ta.tile) * ta.tsq : s0, tp = tiled ? (s0 / ta.tile) * ta.tsp : s0,
                      tj = tiled ? (s0 / ta.tile) * ta.tsj : s0;
        const T* qc = q ? q + tq : q;
        T* pc = poses ? poses + tp : poses;
        T* jc = jac ? jac + tj : jac;
        if (jf && jf->fk) {
            const int per_lane = per_lane_env ? per_lane_env : 1;
            const hipFunction_t jit = per_lane > 1 && jf->fk_stride ? jf->fk_stride : jf->fk;
            const unsigned gx = jit == jf->fk ? grid.x : (grid.x + per_lane - 1) / per_lane;
            int64_t cc = c;
            void* args[] = {(void*)&qc, (void*)&ldq, (void*)&cc, (void*)&pc, (void*)&ldp, (void*)&jc, (void*)&ldj,
                            (void*)&tl};
            // (specialised kernels keep branch frames in registers: no dynamic LDS)
            const unsigned lds = fk_lds_env >= 0 ? (unsigned)fk_lds_env : jit == jf->fk ? kFkLds : 0u;
            const hipError_t e = hipModuleLaunchKernel(jit, gx, 1, 1, block.x, 1, 1, lds, st, args, nullptr);
            if (e != hipSuccess) return e;
            continue;
        }
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
                                     int64_t, T*, int64_t, T*, int64_t, const TileArgs&, const JitFns*,      \
                                     hipStream_t);                                                           \
    template hipError_t launch_pose_residual<T>(const T*, int64_t, const T*, int64_t, int64_t, int, T*, int64_t, \
                                                hipStream_t);
KIN_INSTANTIATE(float)
KIN_INSTANTIATE(double)

}  // namespace kinhip
