// Issue cost of the cross-lane moves the collision-IK kernels use, one wave per SIMD (1024 waves of 64 on
// 256 CUs): 16 independent chains of (move, add) per iteration, the move a plain v_mov, a DPP quad_perm, a DPP
// row_newbcast:l (the row_bcast16 broadcast), a v_readlane + s_add, or a ds_bpermute; plus one dependent
// chain of each (latency).  hipcc --offload-arch=gfx950 -O3 tools/dpp_probe.hip -o /tmp/dpp_probe && /tmp/dpp_probe
#include <hip/hip_runtime.h>

#include <cstdio>

template <int CTL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTL, 0xF, 0xF, false));
}

template <int MODE, int CH>
__global__ __launch_bounds__(256) void k_probe(float* out, float a, int n) {
    float x[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) x[k] = threadIdx.x * 1e-3f + k;
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            float m;
            if constexpr (MODE == 0) m = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(0) + __float_as_int(x[k]));
            else if constexpr (MODE == 1) m = dpp<0x1B>(x[k]);          // quad_perm [3,2,1,0]
            else if constexpr (MODE == 2) m = dpp<0x155>(x[k]);  // row_newbcast:5
            else if constexpr (MODE == 3) m = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x[k]), k & 63));
            else m = __int_as_float(__builtin_amdgcn_ds_bpermute((int)((threadIdx.x ^ 1) * 4), __float_as_int(x[k])));
            x[k] = m + a;
        }
    }
    float s = 0;
#pragma unroll
    for (int k = 0; k < CH; ++k) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int MODE, int CH>
static float run(float* out, int n) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL((k_probe<MODE, CH>), dim3(256), dim3(256), 0, 0, out, 1e-7f, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return best * 1e6f / (float)(n * CH);  // ns per (move + add) pair
}

int main() {
    float* out;
    hipMalloc(&out, 1024 * 256 * sizeof(float));
    const int n = 4096;
    const char* names[] = {"v_mov (+readfirstlane 0)", "dpp quad_perm", "dpp row_newbcast", "v_readlane", "ds_bpermute"};
    float t16[5] = {run<0, 16>(out, n), run<1, 16>(out, n), run<2, 16>(out, n), run<3, 16>(out, n), run<4, 16>(out, n)};
    float t1[5] = {run<0, 1>(out, n), run<1, 1>(out, n), run<2, 1>(out, n), run<3, 1>(out, n), run<4, 1>(out, n)};
    for (int m = 0; m < 5; ++m)
        printf("%-26s 16 chains %.2f ns per (move, add)   1 chain %.2f ns per (move, add)\n", names[m], t16[m], t1[m]);
    hipFree(out);
    return 0;
}
