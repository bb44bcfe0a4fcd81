// Tiled-SoA layout probe (no kinematics): the FK+J fp32 byte pattern (read 8
// rows, write 60 rows per configuration) in three layouts --
//   soa      element (i, r) at r*ld + i            (Julia Matrix(N, rows); ld = N + 256)
//   tile<T>  element (i, r) at (i/T)*rows*T + r*T + i%T   (Julia Array(T, rows, N/T))
//   fill     one contiguous write stream of the same bytes (ceiling)
// Build: hipcc -O3 --offload-arch=gfx950 tools/tile_probe.hip -o kinematics.jl_amd/lib/tile_probe
// Run:   tile_probe <rows R> [log2 sizes, e.g. 20,22,24]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void p_soa(const float* __restrict__ q, float* __restrict__ out, long n, int R, long ld) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float a = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) a += q[r * ld + i];
    for (int r = 0; r < R; ++r) __builtin_nontemporal_store(a + r, out + (long)r * ld + i);
}

template <int T, bool NT>
__global__ void p_tile(const float* __restrict__ q, float* __restrict__ out, long n, int R) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const long t = i / T, e = i % T;
    const float* qt = q + t * 8 * T + e;
    float* ot = out + t * (long)R * T + e;
    float a = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) a += qt[r * T];
    for (int r = 0; r < R; ++r) {
        if (NT) __builtin_nontemporal_store(a + r, ot + (long)r * T);
        else ot[(long)r * T] = a + r;
    }
}

__global__ void p_tile_rt(const float* __restrict__ q, float* __restrict__ out, long n, int R, long T, long tstride,
                          long qstride) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const long t = i / T, e = i % T;
    const float* qt = q + t * qstride + e;
    float* ot = out + t * tstride + e;
    float a = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) a += qt[r * T];
    for (int r = 0; r < R; ++r) __builtin_nontemporal_store(a + r, ot + (long)r * T);
}

__global__ void p_fill(float4* __restrict__ out, long m4) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m4) out[i] = float4{1, 2, 3, 4};
}

int main(int argc, char** argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 60;  // output rows per configuration
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // sizes: argv[2] = comma-separated log2 sizes (default 20,22)
    std::vector<long> sizes;
    for (const char* p = argc > 2 ? argv[2] : "20,22"; *p;) {
        sizes.push_back(1L << strtol(p, (char**)&p, 10));
        if (*p == ',') ++p;
    }
    for (long n : sizes) {
        const long ldp = n + 8192;
        float *q, *out;
        CK(hipMalloc(&q, 8 * ldp * 4));
        CK(hipMalloc(&out, (long)R * ldp * 4));
        CK(hipMemset(q, 0, 8 * ldp * 4));
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
            printf("{\"n\": %ld, \"probe\": \"%s\", \"us\": %.2f, \"GBs\": %.1f}\n", n, name, s * 1e6, bytes / s / 1e9);
        };
        const double bytes = (8.0 + R) * n * 4;
        const unsigned g = n / 256;
        char nm[128];
        for (long T : {2048L, 4096L, 8192L, 16384L, 65536L, 262144L}) {
            for (long pad : {0L, 256L}) {
                const long ts = R * T + pad, qs = 8 * T + pad;
                if ((n / T) * ts > R * ldp || (n / T) * qs > 8 * ldp) continue;
                snprintf(nm, sizeof nm, "tile_rt T=%ld tilepad=%ld", T, pad);
                timeit(nm, bytes, [&] { p_tile_rt<<<g, 256>>>(q, out, n, R, T, ts, qs); });
            }
        }
        for (long pad : {0L, 64L, 256L, 512L, 4096L + 256L}) {
            const long ld = n + pad;
            if (ld > ldp) continue;
            snprintf(nm, sizeof nm, "soa_nt ld=n+%ld", pad);
            timeit(nm, bytes, [&] { p_soa<<<g, 256>>>(q, out, n, R, ld); });
        }
        for (int rep = 0; rep < 1; ++rep) {
            timeit("soa_pad256_nt", bytes, [&] { p_soa<<<g, 256>>>(q, out, n, R, ldp); });
            timeit("tile64_nt", bytes, [&] { p_tile<64, true><<<g, 256>>>(q, out, n, R); });
            timeit("tile64_plain", bytes, [&] { p_tile<64, false><<<g, 256>>>(q, out, n, R); });
            timeit("tile256_nt", bytes, [&] { p_tile<256, true><<<g, 256>>>(q, out, n, R); });
            timeit("tile256_plain", bytes, [&] { p_tile<256, false><<<g, 256>>>(q, out, n, R); });
            timeit("tile1024_nt", bytes, [&] { p_tile<1024, true><<<g, 256>>>(q, out, n, R); });
            timeit("tile4096_nt", bytes, [&] { p_tile<4096, true><<<g, 256>>>(q, out, n, R); });
            timeit("fill_contig_60n", (double)R * n * 4, [&] { p_fill<<<R * n / 4 / 256, 256>>>((float4*)out, R * n / 4); });
        }
        CK(hipFree(q));
        CK(hipFree(out));
    }
    return 0;
}
