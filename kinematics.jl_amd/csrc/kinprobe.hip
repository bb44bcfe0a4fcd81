// kinprobe.hip -- measurement probe (not part of the engine's C-ABI): the HBM access pattern of a
// kernel's inputs and outputs with no arithmetic, so bench.py can print each leg's ceiling from the
// same run ("frac_of_pattern" = probe time / kernel time).  The probe addresses memory exactly as the
// kernels do (kinhip_device.h, kinhip_fk_dev.h): one buffer descriptor per row (ld_soa / st_soa; the
// collision kernels' soffset form sto_soa for their outputs), a 32-bit lane byte offset, the tile of a
// workgroup from a uniform 32-bit divide (Tiling::tile_blocks), 256-lane workgroups (or 128 / 64), non-temporal
// stores, compile-time row counts, and -- for batches of 2^23 and more, like launch_fk's specialised
// kernel -- the grid-strided form with the next unit's loads issued before this unit's stores.
// Element (config i, row r) lives at (i / tile) * rows * tile + r * tile + i % tile (tiled SoA,
// kin_plan_run_tiled) or at r * ld + i (plain SoA, tile = 0).  Built into lib/libkinprobe.so.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kinhip_device.h"

namespace kinhip {
namespace {
typedef unsigned int u32x4 __attribute__((__vector_size__(16)));

template <int RI>
__device__ __forceinline__ float probe_load(const float* __restrict__ q, int64_t ldq, uint32_t off) {
    float v[RI];
#pragma unroll
    for (int r = 0; r < RI; ++r) v[r] = ld_soa(q, r, ldq, off);
    float a = 0.0f;
#pragma unroll
    for (int r = 0; r < RI; ++r) a += v[r];
    return a;
}

template <int RO, bool SOFF>
__device__ __forceinline__ void probe_store(float* __restrict__ out, int64_t ldo, uint32_t off, float a) {
#pragma unroll
    for (int r = 0; r < RO; ++r) {
        if constexpr (SOFF) sto_soa(out, r, ldo, off, a + (float)r);
        else st_soa(out, r, ldo, off, a + (float)r);
    }
}

// one configuration per lane (k_fk / k_coll at batches below 2^23)
template <int RI, int RO, bool SOFF>
__global__ __launch_bounds__(256) void p_pattern(const float* __restrict__ q, int64_t ldq, float* __restrict__ out,
                                                 int64_t ldo, int64_t n, Tiling tl) {
    const uint32_t b = blockIdx.x, tid = threadIdx.x, B = blockDim.x;
    if ((uint64_t)b * B + tid >= (uint64_t)n) return;
    const uint32_t t = b / tl.tile_blocks;
    q += (int64_t)t * tl.tsq;
    out += (int64_t)t * tl.tsp;
    const uint32_t off = ((b - t * tl.tile_blocks) * B + tid) * 4u;
    probe_store<RO, SOFF>(out, ldo, off, probe_load<RI>(q, ldq, off));
}

// grid-strided units of 256 configurations, the next unit's loads in flight (fk_body<..., true>)
template <int RI, int RO, bool SOFF>
__global__ __launch_bounds__(256) void p_pattern_strided(const float* __restrict__ q, int64_t ldq,
                                                         float* __restrict__ out, int64_t ldo, int64_t n, Tiling tl) {
    const uint32_t tid = threadIdx.x, B = blockDim.x, units = (uint32_t)((n + B - 1) / B);
    uint32_t b = blockIdx.x;
    if (b >= units) return;
    auto addr = [&](uint32_t u, const float*& qb, float*& ob) {
        const uint32_t t = u / tl.tile_blocks;
        qb = q + (int64_t)t * tl.tsq;
        ob = out + (int64_t)t * tl.tsp;
        return ((u - t * tl.tile_blocks) * B + tid) * 4u;
    };
    const float* qb;
    float* ob;
    uint32_t off = addr(b, qb, ob);
    float a = (uint64_t)b * B + tid < (uint64_t)n ? probe_load<RI>(qb, ldq, off) : 0.0f;
    for (;;) {
        const uint32_t bn = b + gridDim.x;
        const bool more = bn < units;
        const float* qn;
        float* on;
        const uint32_t offn = more ? addr(bn, qn, on) : 0u;
        const float an = more && (uint64_t)bn * B + tid < (uint64_t)n ? probe_load<RI>(qn, ldq, offn) : 0.0f;
        if ((uint64_t)b * B + tid < (uint64_t)n) probe_store<RO, SOFF>(ob, ldo, off, a);
        if (!more) break;
        b = bn; off = offn; ob = on; a = an;
    }
}

// the same bytes with the outputs staged through LDS: each lane writes its RO values into an [RO][B] LDS
// block, then every wave writes whole rows, 16 bytes per lane (buffer_store_dwordx4: one instruction
// covers 4 x 64 consecutive configurations of a row instead of 64) -- what an LDS-staged store path in
// k_fk would emit.  Rows must be 16-byte aligned (ld % 4 == 0, tile % 4 == 0).
template <int RI, int RO>
__global__ __launch_bounds__(256) void p_pattern_x4(const float* __restrict__ q, int64_t ldq, float* __restrict__ out,
                                                    int64_t ldo, int64_t n, Tiling tl) {
    extern __shared__ float stage[];  // [RO][B]
    const uint32_t b = blockIdx.x, tid = threadIdx.x, B = blockDim.x;
    const uint32_t t = b / tl.tile_blocks;
    q += (int64_t)t * tl.tsq;
    out += (int64_t)t * tl.tsp;
    const uint32_t i0 = (b - t * tl.tile_blocks) * B;  // first configuration of the block (in its tile)
    const bool valid = (uint64_t)b * B + tid < (uint64_t)n;
    const float a = valid ? probe_load<RI>(q, ldq, (i0 + tid) * 4u) : 0.0f;
#pragma unroll
    for (int r = 0; r < RO; ++r) stage[r * B + tid] = a + (float)r;
    __syncthreads();
    const uint32_t w = tid >> 6, l = tid & 63u, nw = B >> 6, per_row = B / 4;  // lanes per row (16 B each)
    const uint64_t left = (uint64_t)n - (uint64_t)b * B;                      // configurations of this block
    for (uint32_t k = w * 64 + l; k < RO * per_row; k += nw * 64) {
        const uint32_t r = k / per_row, c = (k - r * per_row) * 4;
        if (c + 4 <= left) {
            const float4 v = *reinterpret_cast<const float4*>(&stage[r * B + c]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), row_rsrc(out + r * ldo),
                                                   (int)((i0 + c) * 4u), 0, KINHIP_STORE_AUX);
        } else {
            for (uint32_t e = c; e < B && e < left; ++e)
                st_soa(out, r, ldo, (i0 + e) * 4u, stage[r * B + e]);
        }
    }
}

template <int RI, int RO, bool SOFF>
int launch_pattern(int64_t n, int64_t tile, int64_t ld, const float* q, float* out, int per_lane, int lds, int blk,
                   hipStream_t st) {
    const bool tiled = tile > 0;
    if (tiled && tile % blk) return -1;
    // tiled arrays: (ntiles, rows, tile) -- a tile of q is RI rows, a tile of out RO rows
    Tiling tl{tiled ? (uint32_t)(tile / blk) : 0xffffffffu, tiled ? RI * tile : 0, tiled ? RO * tile : 0, 0, 0};
    const int64_t ldr = tiled ? tile : ld;
    if ((uint64_t)(tiled ? tile : n) * 4u >= (1ull << 31)) return -1;  // 32-bit lane offsets
    if (SOFF && (uint64_t)(RO * ldr + (tiled ? tile : n)) * 4u >= (1ull << 31)) return -1;
    const unsigned units = (unsigned)((n + blk - 1) / blk);
    // lds: dynamic LDS bytes per workgroup, unused -- it only caps how many workgroups a CU holds (the
    // probe's few registers would otherwise keep more waves in flight than any kernel it bounds)
    if (per_lane > 1)
        hipLaunchKernelGGL((p_pattern_strided<RI, RO, SOFF>), dim3((units + per_lane - 1) / per_lane), dim3(blk),
                           (size_t)lds, st, q, ldr, out, ldr, n, tl);
    else if (per_lane < 0) {  // (-1: the LDS-staged 16-byte row stores; lds is the staging block, at least RO * blk * 4)
        if (SOFF || ldr % 4 || (size_t)RO * blk * 4 > 65536) return -1;
        const size_t need = (size_t)RO * blk * 4;
        hipLaunchKernelGGL((p_pattern_x4<RI, RO>), dim3(units), dim3(blk), (size_t)lds > need ? (size_t)lds : need, st,
                           q, ldr, out, ldr, n, tl);
    } else
        hipLaunchKernelGGL((p_pattern<RI, RO, SOFF>), dim3(units), dim3(blk), (size_t)lds, st, q, ldr, out, ldr, n, tl);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}

}  // namespace
}  // namespace kinhip

// rows_in / rows_out: (8, 60) FK + 6x8 J + pose (k_fk), (8, 126) 14 sphere distances + gradients
// (k_coll, soffset-addressed outputs), (12, 126) the same with 4 scene columns in (k_coll_scene).  Plain rows (tile = 0) ld >= n elements apart; tiled: ld = tile.
// per_lane > 1: the grid-strided form with that many units per workgroup; -1: the LDS-staged 16-byte row stores
// (p_pattern_x4, a layout experiment for k_fk).  lds: dynamic LDS bytes per
// workgroup (0..65536) to cap the waves in flight per CU; blk: lanes per workgroup (64..256, a power of 2).
extern "C" __attribute__((visibility("default"))) int kinprobe_pattern4(int rows_in, int rows_out, int64_t n,
                                                                        int64_t tile, int64_t ld, int per_lane,
                                                                        int lds, int blk, const float* q, float* out,
                                                                        void* stream) {
    if (n <= 0 || n >= (int64_t(1) << 30) || tile < 0 || (tile > 0 ? ld != tile : ld < n) || per_lane < -1 || per_lane == 0 ||
        lds < 0 || lds > 65536 || (blk != 64 && blk != 128 && blk != 256))
        return -1;
    const hipStream_t st = (hipStream_t)stream;
    if (rows_in == 8 && rows_out == 60)
        return kinhip::launch_pattern<8, 60, false>(n, tile, ld, q, out, per_lane, lds, blk, st);
    if (rows_in == 8 && rows_out == 126)
        return kinhip::launch_pattern<8, 126, true>(n, tile, ld, q, out, per_lane, lds, blk, st);
    if (rows_in == 12 && rows_out == 126)  // (the f2 door sweep: q + the scene columns in)
        return kinhip::launch_pattern<12, 126, true>(n, tile, ld, q, out, per_lane, lds, blk, st);
    return -2;
}

extern "C" __attribute__((visibility("default"))) int kinprobe_pattern3(int rows_in, int rows_out, int64_t n,
                                                                        int64_t tile, int64_t ld, int per_lane,
                                                                        int lds, const float* q, float* out,
                                                                        void* stream) {
    return kinprobe_pattern4(rows_in, rows_out, n, tile, ld, per_lane, lds, 256, q, out, stream);
}
