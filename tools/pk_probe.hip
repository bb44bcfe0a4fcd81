// Issue cost of packed vs scalar fp32 FMA for one wave per SIMD (1024 waves of 64 on 256 CUs) and for
// two / four: 8 independent accumulator chains, 4096 iterations.  hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize
// tools/pk_probe.hip -o /tmp/pk_probe && /tmp/pk_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float float2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_scalar(float* out, float a, float b, int n) {
    float x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = threadIdx.x * 1e-3f + k;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = __builtin_fmaf(x[k], a, b);
    }
    float s = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_packed(float* out, float a, float b, int n) {
    float2v x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = float2v{threadIdx.x * 1e-3f + 2 * k, threadIdx.x * 1e-3f + 2 * k + 1};
    const float2v av = {a, a}, bv = {b, b};
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = __builtin_elementwise_fma(x[k], av, bv);
    }
    float s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += x[k].x + x[k].y;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    float* out;
    hipMalloc(&out, 4 * 1024 * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int n = 4096;
    for (int waves_per_simd = 1; waves_per_simd <= 4; waves_per_simd *= 2) {
        const int blocks = 256 * waves_per_simd;  // 4 waves per block, one per SIMD
        for (int pk = 0; pk < 2; ++pk) {
            float best = 1e30f;
            for (int r = 0; r < 5; ++r) {
                hipEventRecord(e0);
                if (pk) hipLaunchKernelGGL(k_packed, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f, n);
                else hipLaunchKernelGGL(k_scalar, dim3(blocks), dim3(256), 0, 0, out, 0.999f, 1e-3f, n);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            // 16 fp32 FMAs per lane-iteration either way
            const double instr = pk ? 8.0 * n : 16.0 * n;
            printf("%d wave(s)/SIMD %s: %.3f ms, %.2f ns per wave-instruction, %.2f ns per lane-FMA slot\n",
                   waves_per_simd, pk ? "v_pk_fma_f32" : "v_fma_f32   ", best, best * 1e6 / instr,
                   best * 1e6 / (16.0 * n));
        }
    }
    hipFree(out);
    return 0;
}
