// Store-pattern ceiling probe (no kinematics): what HBM delivers for the FK+J
// output shapes, to separate memory-pattern limits from kernel compute.
// Build: hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o gpurun_out/store_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

// P1: one config per lane, read 8 rows, write R rows (4 B per lane per row)
// rows `ld` elements apart (ld = n: dense; ld = n + 256: the bench's padded rows)
template <bool NT>
__global__ void p_narrow(const float* __restrict__ q, float* __restrict__ out, long n, int R, long ld) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) a += q[r * ld + i];
    for (int r = 0; r < R; ++r) {
        float v = a + r;
        if (NT) __builtin_nontemporal_store(v, out + (long)r * ld + i);
        else out[(long)r * ld + i] = v;
    }
}
// P2: four consecutive configs per lane (16 B per lane per row, 1 KB per row per wave)
template <bool NT>
__global__ void p_vec4(const float4* __restrict__ q, float4* __restrict__ out, long n4, int R) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n4) return;
    float4 a = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < 8; ++r) { float4 x = q[r * n4 + i]; a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w; }
    for (int r = 0; r < R; ++r) {
        float4 v = {a.x + r, a.y + r, a.z + r, a.w + r};
        typedef float f4 __attribute__((ext_vector_type(4)));
        f4 w = {v.x, v.y, v.z, v.w};
        f4* p = reinterpret_cast<f4*>(out + (long)r * n4 + i);
        if (NT) __builtin_nontemporal_store(w, p);
        else *p = w;
    }
}
// P3: contiguous fill of R*n floats, 16 B per lane
__global__ void p_fill(float4* __restrict__ out, long m4) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m4) out[i] = float4{1, 2, 3, 4};
}

int main() {
    const long n = 1 << 20;
    const int R = 60;
    float *q, *out;
    const long ldp = n + 256;
    CK(hipMalloc(&q, 8 * ldp * 4));
    CK(hipMalloc(&out, (long)R * ldp * 4));
    CK(hipMemset(q, 0, 8 * ldp * 4));
    float* out2;
    CK(hipMalloc(&out2, 126L * n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, double bytes, auto launch) {
        for (int w = 0; w < 10; ++w) launch();
        hipDeviceSynchronize();
        const int K = 100;
        hipEventRecord(e0);
        for (int k = 0; k < K; ++k) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double s = ms / 1e3 / K;
        printf("{\"probe\": \"%s\", \"us\": %.2f, \"GBs\": %.1f}\n", name, s * 1e6, bytes / s / 1e9);
    };
    const double bytes = (8.0 + R) * n * 4;
    for (int rep = 0; rep < 2; ++rep) {
        timeit("narrow_60rows_plain", bytes, [&] { p_narrow<false><<<n / 256, 256>>>(q, out, n, R, n); });
        timeit("narrow_60rows_nt", bytes, [&] { p_narrow<true><<<n / 256, 256>>>(q, out, n, R, n); });
        timeit("narrow_60rows_plain_pad256", bytes, [&] { p_narrow<false><<<n / 256, 256>>>(q, out, n, R, ldp); });
        timeit("narrow_60rows_nt_pad256", bytes, [&] { p_narrow<true><<<n / 256, 256>>>(q, out, n, R, ldp); });
        timeit("vec4_60rows_plain", bytes, [&] { p_vec4<false><<<n / 4 / 256, 256>>>((float4*)q, (float4*)out, n / 4, R); });
        timeit("vec4_60rows_nt", bytes, [&] { p_vec4<true><<<n / 4 / 256, 256>>>((float4*)q, (float4*)out, n / 4, R); });
        timeit("narrow_126rows_nt (config-5 grads: 8 in, 14 + 112 out)", (8.0 + 126) * n * 4,
               [&] { p_narrow<true><<<n / 256, 256>>>(q, out2, n, 126, n); });
        timeit("fill_contig_60n", (double)R * n * 4, [&] { p_fill<<<R * n / 4 / 256, 256>>>((float4*)out, R * n / 4); });
    }
    return 0;
}
