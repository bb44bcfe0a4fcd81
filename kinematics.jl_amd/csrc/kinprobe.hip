// kinprobe.hip -- measurement probe (not part of the engine's C-ABI): the HBM access pattern of a
// kernel's inputs and outputs with no arithmetic, so bench.py can print each leg's ceiling from the
// same run ("frac_of_pattern" = probe time / kernel time).  Element (config i, row r) of an array
// lives at (i / tile) * rows * tile + r * tile + i % tile (tiled SoA, kin_plan_run_tiled) or at
// r * ld + i (plain SoA, tile = 0); every lane reads rows_in rows of q and writes rows_out rows with
// non-temporal stores, exactly like k_fk / k_coll.  Built into lib/libkinprobe.so by the Makefile.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__global__ __launch_bounds__(256) void p_pattern(const float* __restrict__ q, float* __restrict__ out, int64_t n,
                                                 int rows_in, int rows_out, int64_t tile, int64_t ldq, int64_t ldo) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t t = tile > 0 ? i / tile : 0, e = tile > 0 ? i % tile : i;
    const float* qt = q + t * rows_in * ldq + e;
    float* ot = out + t * rows_out * ldo + e;
    float a = 0.0f;
    for (int r = 0; r < rows_in; ++r) a += qt[r * ldq];
    for (int r = 0; r < rows_out; ++r) __builtin_nontemporal_store(a + (float)r, ot + (int64_t)r * ldo);
}

}  // namespace

// plain rows (tile = 0) ld elements apart (ld >= n: a padded row stride); tiled: ld is the tile
extern "C" __attribute__((visibility("default"))) int kinprobe_pattern_ld(int rows_in, int rows_out, int64_t n,
                                                                          int64_t tile, int64_t ld, const float* q,
                                                                          float* out, void* stream) {
    if (n <= 0 || rows_in < 0 || rows_out < 1 || tile < 0 || (tile > 0 ? ld != tile : ld < n)) return -1;
    hipLaunchKernelGGL(p_pattern, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, q, out, n,
                       rows_in, rows_out, tile, ld, ld);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}

extern "C" __attribute__((visibility("default"))) int kinprobe_pattern(int rows_in, int rows_out, int64_t n,
                                                                       int64_t tile, const float* q, float* out,
                                                                       void* stream) {
    return kinprobe_pattern_ld(rows_in, rows_out, n, tile, tile > 0 ? tile : n, q, out, stream);
}
